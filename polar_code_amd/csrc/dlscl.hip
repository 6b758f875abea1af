// dlscl.hip -- DL-SCL bit-flip retry rounds on the device (dlscl/flip.py:65-141).
//
// The retry loop of decode_with_retries runs over a compacted list of the frames whose
// baseline SCL best candidate fails the CRC.  Each frame keeps, in an "entry" slot, the
// state the reference threads through its loop (flip.py:110-136): the reference bits, the
// decision LLRs L0 of the best path, and the set of tried indices.  One round is
//   dl_select_kernel  q = |L0| @ beta (or |L0|), flip = argmin over untried (q, index),
//                     force vector = reference prefix + flipped bit (flip.py:30-34)
//   decode            the SCL kernel on the live entries (LLR row indirection, forced bits)
//   replay_kernel     L0 of the attempt's best path (flip.py:127-132), recomputed from its bits
//   dl_update_kernel  final-attempt bookkeeping, CRC stop rule, compaction of the survivors
// Frames never leave the GPU.  The live counts stay on the device: every round is enqueued
// with grids sized for the first round, and waves past the live count exit at once.
//
// Why a replay instead of the decoder's history: the decision LLR of a path at info phase
// j (scl.py:158,166) is a function of the channel LLRs and the path's own earlier bits only
// (lazy copies share, never alter, ancestors' values).  With the final bits known, every
// leaf LLR follows top-down, level by level, through the same f/g operations -- bit-identical
// values at ~1/15 of a decode, and the decode itself keeps the occupancy of the plain kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "polar_scl.h"
#include "scl_device.h"
#include "scl_kernels.h"

#pragma clang fp contract(off)

namespace {

using pscl::f_minsum;
using pscl::g_node;
using pscl::polar_transform64;

// monotone map of an fp64 to uint64 (total order of non-NaN values, -0 == +0)
__device__ __forceinline__ uint64_t order_key(double q) {
    if (q == 0.0) q = 0.0;
    const uint64_t u = (uint64_t)__double_as_longlong(q);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}

using pscl::wave_sum;

// failing baseline frames of a chunk -> act[] (entry e holds frame base + f); list[e] = e.
// One atomic per 1024-thread block.
__global__ void __launch_bounds__(1024) dl_compact_kernel(const uint8_t* __restrict__ flags, int64_t B, int64_t base,
                                                          int64_t* __restrict__ act, int32_t* __restrict__ list,
                                                          int32_t* __restrict__ count) {
    __shared__ int wcnt[16];
    __shared__ int bbase;
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool failing = f < B && !(flags[f] & PSCL_FLAG_CRC_PASS);
    const uint64_t m = __ballot(failing);
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
            const int c = wcnt[w];
            wcnt[w] = acc;
            acc += c;
        }
        bbase = acc ? atomicAdd(count, acc) : 0;
    }
    __syncthreads();
    if (failing) {
        const int pos = bbase + wcnt[wave] + __popcll(m & ((1ULL << lane) - 1ULL));
        act[pos] = base + f;
        list[pos] = pos;
    }
}

__global__ void __launch_bounds__(256) iota64_kernel(int64_t* out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = i;
}

// entry reference bits = the frame's baseline best bits
__global__ void __launch_bounds__(256) dl_gather_kernel(const uint64_t* __restrict__ best, const int64_t* __restrict__ act,
                                                        const int32_t* __restrict__ count, int W,
                                                        uint64_t* __restrict__ ref) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= *count) return;
    for (int w = 0; w < W; ++w) ref[e * W + w] = best[act[e] * W + w];
}

// one wavefront per entry: leaf LLRs of the entry's path (bits given), written at its info
// positions.  LDS: two 128-double level buffers per wave.
__global__ void __launch_bounds__(256) replay_kernel(const pscl_replay_params R, int64_t cap) {
    __shared__ double lvl[4][2][PSCL_FAST_N];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + wave;
    if (b >= *R.count || b >= cap) return;
    const int N = R.N, K = R.K, W = R.W;
    const int e = R.list ? R.list[b] : (int)b;
    const int64_t row = R.act[e];
    double* cur = lvl[wave][0];
    double* nxt = lvl[wave][1];
    for (int p = lane; p < N; p += 64) {
        if (R.rm_E == 0) cur[p] = R.llr[row * N + p];
        else cur[p] = pscl::nr_stage(R.llr + row * R.rm_E, R.rm_src[p], R.rm_E, N);
    }
    // the path's u: frozen 0, info position p carries bit j = #info positions below p
    const uint64_t* bw = R.bits + (R.bits_by_row ? row : b) * W;
    uint64_t u[2] = {0, 0};
    int jpos[2] = {-1, -1};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int p = lane + 64 * h;
        bool bit = false;
        if (p < N && ((R.info_mask[h] >> lane) & 1ULL)) {
            const int j = (h ? __popcll(R.info_mask[0]) : 0) + __popcll(R.info_mask[h] & ((1ULL << lane) - 1ULL));
            jpos[h] = j;
            bit = (bw[j >> 6] >> (j & 63)) & 1ULL;
        }
        u[h] = __ballot(bit);
    }
    pscl::wave_lds_fence();
    // level d -> d+1: node k' of width w2 at flat position p' = k' w2 + i; its parent's
    // halves are a = lvl_d[(k'>>1) 2 w2 + i], b = a's partner + w2 (polar.py:122-127)
    for (int d = 0; d < R.n; ++d) {
        // w2 = N >> (d + 1) = 2^lw2: node index and offset by shift and mask (a runtime
        // integer division here cost more VALU than the f/g work of the whole replay)
        const int lw2 = R.n - d - 1, w2 = 1 << lw2;
        for (int p2 = lane; p2 < N; p2 += 64) {
            const int k2 = p2 >> lw2, i = p2 & (w2 - 1);
            const int pa = ((k2 >> 1) << (lw2 + 1)) + i;
            const double a = cur[pa], bb = cur[pa + w2];
            double v;
            if (!(k2 & 1)) {
                v = f_minsum(a, bb);
            } else {  // partial sums of the left sibling u[(k2-1) w2, k2 w2)
                const int lo = (k2 - 1) * w2;
                const uint64_t word = u[lo >> 6] >> (lo & 63);
                const uint64_t chunk = w2 >= 64 ? word : (word & ((1ULL << w2) - 1ULL));
                v = g_node(a, bb, (uint32_t)(polar_transform64(chunk) >> i) & 1u);
            }
            nxt[p2] = v;
        }
        pscl::wave_lds_fence();
        double* t = cur;
        cur = nxt;
        nxt = t;
    }
    double* out = R.out + (int64_t)e * K;
#pragma unroll
    for (int h = 0; h < 2; ++h)
        if (jpos[h] >= 0) out[jpos[h]] = cur[lane + 64 * h];
}

// wavefronts over live entries, beta staged in LDS: choose the flip index, build the force
// words (persistent grid)
__global__ void __launch_bounds__(256) dl_select_kernel(const pscl_dl_params D) {
    extern __shared__ double sbeta[];
    const int K = D.K, W = D.W;
    if (D.beta) {
        for (int i = threadIdx.x; i < K * K; i += blockDim.x) sbeta[i] = D.beta[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int n = *D.n;
    for (int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); b < n; b += (int64_t)gridDim.x * 4) {
        const int e = D.list[b];
        const double* a = D.al0 + (int64_t)e * K;
        const uint64_t t0 = D.tried[2 * e], t1 = D.tried[2 * e + 1];
        uint64_t bk = ~0ULL;
        int bj = 0x7fffffff;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = lane + 64 * h;
            if (j < K) {
                double q;
                if (D.beta) {  // q = abs_l0 @ beta (flip.py:104-106), summed in index order
                    q = 0.0;
                    for (int k = 0; k < K; ++k) q = q + fabs(a[k]) * sbeta[k * K + j];
                } else {
                    q = fabs(a[j]);  // flip.py:107
                }
                const bool seen = ((h ? t1 : t0) >> (j & 63)) & 1ULL;
                const uint64_t key = seen ? ~0ULL : order_key(q);
                if (key < bk) {  // h = 0 visited first: ties keep the lower index
                    bk = key;
                    bj = j;
                }
            }
        }
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {  // wave argmin of (key, index)
            const uint64_t ok = pscl::shfl_u64(bk, lane ^ s);
            const int oj = __shfl(bj, lane ^ s);
            if (ok < bk || (ok == bk && oj < bj)) {
                bk = ok;
                bj = oj;
            }
        }
        if (lane == 0) {
            const int idx = bj;  // an untried index exists: rounds <= min(retries, K)
            const int nt = D.ntried[e];
            const int64_t f = D.act[e];
            if (idx >= 64) D.tried[2 * e + 1] = t1 | (1ULL << (idx - 64)); else D.tried[2 * e] = t0 | (1ULL << idx);
            D.ntried[e] = nt + 1;
            if (D.tried_out) D.tried_out[f * D.tried_stride + nt] = idx;
            D.fidx[b] = f;
            // _force_vector (flip.py:30-34): bits [0, idx) = reference, bit idx flipped, rest free
            const uint64_t* ref = D.ref + (int64_t)e * W;
            uint64_t* fr = D.force + b * 2 * W;
            for (int w = 0; w < W; ++w) {
                const int lo = 64 * w;
                const int nb = idx - lo + 1;  // bits of this word in [0, idx]
                const uint64_t mask = nb <= 0 ? 0ULL : (nb >= 64 ? ~0ULL : ((1ULL << nb) - 1ULL));
                uint64_t val = ref[w] & mask;
                if (idx >= lo && idx < lo + 64) val ^= 1ULL << (idx - lo);
                fr[w] = mask;
                fr[W + w] = val;
            }
        }
    }
}

// one thread per live entry: record the attempt, stop on CRC pass or retry budget, carry
// the attempt's best bits into the entry state (flip.py:123-136); survivors appended with
// one atomic per wavefront
__global__ void __launch_bounds__(256) dl_update_kernel(const pscl_dl_params D) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int n = *D.n;
    const int lane = threadIdx.x & 63;
    const int W = D.W;
    bool more = false;
    int e = 0;
    if (b < n) {
        e = D.list[b];
        const int64_t f = D.act[e];
        const uint8_t fl = D.oflags[b];
        const int nt = D.ntried[e];
        more = !(fl & PSCL_FLAG_CRC_PASS) && nt < D.rounds;
        for (int w = 0; w < W; ++w) {
            const uint64_t v = D.ob[b * W + w];
            D.best[f * W + w] = v;
            if (more) D.ref[(int64_t)e * W + w] = v;
        }
        D.flags[f] = fl;
        if (D.attempts) D.attempts[f] = nt + 1;
    }
    if (b == 0 && D.counters && n > 0)
        atomicAdd(reinterpret_cast<unsigned long long*>(D.counters) + PSCL_CNT_RETRIES, (unsigned long long)n);
    const uint64_t m = __ballot(more);
    if (!m) return;
    const int leader = __builtin_ctzll(m);
    int base = 0;
    if (lane == leader) base = atomicAdd(D.next_count, __popcll(m));
    base = __shfl(base, leader);
    if (more) D.next_list[base + __popcll(m & ((1ULL << lane) - 1ULL))] = e;
}

// FER/BER statistics of the final results against the transmitted words: wavefront sums,
// then one atomic per counter per 1024-thread block
__global__ void __launch_bounds__(1024) dl_count_kernel(const uint64_t* __restrict__ best, const uint8_t* __restrict__ flags,
                                                        const uint64_t* __restrict__ ref, int64_t B, int W, int k_payload,
                                                        int64_t* counters) {
    __shared__ int part[16][4];
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned long long* C = reinterpret_cast<unsigned long long*>(counters);
    if (f == 0) atomicAdd(C + PSCL_CNT_FRAMES, (unsigned long long)B);
    int v[4] = {0, 0, 0, 0};  // frame errors, bit errors, payload frame errors, payload bit errors
    if (f < B) {
        const uint64_t d0 = best[f * W] ^ ref[f * W];
        const uint64_t d1 = W > 1 ? best[f * W + 1] ^ ref[f * W + 1] : 0ULL;
        const int kp = k_payload;
        const uint64_t pm0 = kp >= 64 ? ~0ULL : ((1ULL << kp) - 1);
        const uint64_t pm1 = kp >= 128 ? ~0ULL : (kp > 64 ? ((1ULL << (kp - 64)) - 1) : 0ULL);
        v[0] = (flags[f] & PSCL_FLAG_CRC_PASS) ? 0 : 1;
        v[1] = __popcll(d0) + __popcll(d1);
        v[3] = __popcll(d0 & pm0) + __popcll(d1 & pm1);
        v[2] = v[3] ? 1 : 0;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = wave_sum(v[i]);
    if (lane == 0)
        for (int i = 0; i < 4; ++i) part[wave][i] = v[i];
    __syncthreads();
    if (threadIdx.x < 4) {
        long long t = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += part[w][threadIdx.x];
        static const int slot[4] = {PSCL_CNT_FRAME_ERR, PSCL_CNT_BIT_ERR, PSCL_CNT_PAYLOAD_ERR, PSCL_CNT_PAYLOAD_BIT};
        if (t) atomicAdd(C + slot[threadIdx.x], (unsigned long long)t);
    }
}

}  // namespace

hipError_t pscl_launch_dl_compact(const uint8_t* flags, int64_t B, int64_t base, int64_t* act, int32_t* list,
                                  int32_t* count, hipStream_t s) {
    const int64_t grid = (B + 1023) / 1024;
    hipLaunchKernelGGL(dl_compact_kernel, dim3((unsigned)grid), dim3(1024), 0, s, flags, B, base, act, list, count);
    return hipGetLastError();
}

hipError_t pscl_launch_iota64(int64_t* out, int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(iota64_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out, n);
    return hipGetLastError();
}

hipError_t pscl_launch_dl_gather(const uint64_t* best, const int64_t* act, const int32_t* count, int64_t cap, int W,
                                 uint64_t* ref, hipStream_t s) {
    if (cap <= 0) return hipSuccess;
    hipLaunchKernelGGL(dl_gather_kernel, dim3((unsigned)((cap + 255) / 256)), dim3(256), 0, s, best, act, count, W, ref);
    return hipGetLastError();
}

hipError_t pscl_launch_replay(const pscl_replay_params& R, int64_t cap, hipStream_t s) {
    if (cap <= 0) return hipSuccess;
    const int64_t grid = (cap + 3) / 4;
    hipLaunchKernelGGL(replay_kernel, dim3((unsigned)grid), dim3(256), 0, s, R, cap);
    return hipGetLastError();
}

hipError_t pscl_launch_dl_select(const pscl_dl_params& D, int64_t cap, hipStream_t s) {
    if (cap <= 0) return hipSuccess;
    int64_t grid = (cap + 3) / 4;
    if (grid > 2048) grid = 2048;
    const int lds = D.beta ? D.K * D.K * 8 : 0;
    hipLaunchKernelGGL(dl_select_kernel, dim3((unsigned)grid), dim3(256), lds, s, D);
    return hipGetLastError();
}

hipError_t pscl_launch_dl_update(const pscl_dl_params& D, int64_t cap, hipStream_t s) {
    if (cap <= 0) return hipSuccess;
    const int64_t grid = (cap + 255) / 256;
    hipLaunchKernelGGL(dl_update_kernel, dim3((unsigned)grid), dim3(256), 0, s, D);
    return hipGetLastError();
}

hipError_t pscl_launch_dl_count(const uint64_t* best, const uint8_t* flags, const uint64_t* ref, int64_t B, int W,
                                int k_payload, int64_t* counters, hipStream_t s) {
    const int64_t grid = (B + 1023) / 1024;
    hipLaunchKernelGGL(dl_count_kernel, dim3((unsigned)grid), dim3(1024), 0, s, best, flags, ref, B, W, k_payload,
                       counters);
    return hipGetLastError();
}
