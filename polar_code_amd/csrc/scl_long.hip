// scl_long.hip -- list decoder for code lengths above 128 (256, 512, 1024), any list size
// L <= 32: decode_scl (dl_scl_polar/polar/scl.py:108-209) accepts any power-of-two N
// (scl.py:25-30); the specialised kernels stop at N = 128 (one or two 64-bit words of decided
// bits in registers, the LLR tree in LDS).  Here one wavefront decodes one frame and the
// per-frame state lives in a global scratch area of its workgroup (L2 / Infinity-Cache
// resident): at N = 1024 and L = 8 the path trees alone are 65 KB per frame.
//
// Same algorithm and bit-exact results as scl_kernels.hip's generic kernel:
//   * LLR tree: per path slot, depths 1..n-1 (node at depth d: N >> d values); depth 0 is the
//     frame's channel row, staged (de-rate-matched when rate matching is on).  Lazy copy: a
//     path only copies its table of per-depth slot indices; at phase phi every path rewrites
//     its own slot at the depths >= start(phi) (successive cancellation is lockstep), reading
//     its parent node from the slot its table names (scl.py:64-78, _ensure_alpha).
//   * decided bits: N bits per path in scratch, double-buffered; survivors copy their parent's
//     words (scl.py:52-62 clone) -- N/64 words each.
//   * partial sums of the g node's left sibling: the Arikan transform of u[phi - w, phi)
//     (w = 2^ctz(phi)): one register word for w <= 64, else w/64 words built in LDS (in-word
//     transforms, then cross-word butterfly stages) -- scl.py:84-99 set_bit, recomputed.
//   * metric: np.logaddexp(0, +-llr) by the bit-exact glibc port (glibc_softplus.h);
//     list: Python's stable sort as a rank count on (metric, 2 * list position + bit).
//   * epilogue: u[info_set], CRC syndrome from the K check columns, best = first CRC pass.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "glibc_softplus.h"
#include "scl_device.h"
#include "scl_kernels.h"

namespace {

using namespace pscl;

constexpr int kMaxLongN = 1024;
constexpr int kMaxXsWords = kMaxLongN / 2 / 64;  // widest left sibling: N/2 bits

// doubles of the path trees: depth 0 (N, one copy) + LMAX slots of depths 1..n-1
__host__ __device__ inline int64_t long_tree_doubles(int N, int lmax) { return (int64_t)N + (int64_t)lmax * (N - 2); }
// offset (doubles) of depth d >= 1, slot s
__device__ __forceinline__ int64_t long_node_off(int N, int lmax, int d, int s) {
    return (int64_t)N + (int64_t)lmax * (N - (N >> (d - 1))) + (int64_t)s * (N >> d);
}
__device__ __forceinline__ int long_slot(uint64_t tab, int d) { return (int)((tab >> (5 * (d - 1))) & 31u); }

// make the wave's global-scratch and LDS stores visible to its own later loads
__device__ __forceinline__ void wave_mem_fence() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// minimum waves per SIMD the register allocation must allow: 8 (64 VGPRs; the plain
// instances fit without spills, the history ones spill a few words).  Measured on MI355X
// (tools/long_bench.py): 7 waves/SIMD at the compiler's ~70 VGPRs -> 8 is 10-11 % faster at
// N = 256..1024, L = 8.  0: the compiler's choice.
#ifndef PSCL_LONG_WAVES_PER_EU
#define PSCL_LONG_WAVES_PER_EU 8
#endif
// The history instances and L = 16 spill 6-10 VGPRs at 64 (scratch: private-memory traffic and
// the per-queue scratch allocation at the first dispatch); they build for one wave fewer (the
// L = 16 history instance for two)
#ifndef PSCL_LONG_SPILL_WAVES_PER_EU
#define PSCL_LONG_SPILL_WAVES_PER_EU 7
#endif
#if PSCL_LONG_WAVES_PER_EU
#define PSCL_LONG_BOUNDS \
    __launch_bounds__(64, (HIST && LMAX == 16) ? PSCL_LONG_SPILL_WAVES_PER_EU - 1 \
                          : (HIST || LMAX == 16) ? PSCL_LONG_SPILL_WAVES_PER_EU : PSCL_LONG_WAVES_PER_EU)
#else
#define PSCL_LONG_BOUNDS __launch_bounds__(64)
#endif

template <int LMAX, bool HIST>
__global__ void PSCL_LONG_BOUNDS scl_long_kernel(const pscl_decode_params P) {
    constexpr int G = 2 * LMAX;  // candidate lanes: path p in lane p, its bit-1 child in lane p + LMAX
    __shared__ uint64_t T[PSCL_EXP_TABLE_WORDS];
    __shared__ uint64_t xsw[LMAX * kMaxXsWords];
    __shared__ uint8_t inv[64];
    __shared__ uint64_t tab_lds[LMAX], xs_lds[LMAX];  // path state read by the element lanes
    __shared__ uint64_t key_lds[64];                  // children's metrics (candidate c = p + LMAX * bit)
    __shared__ uint32_t kt_lds[64];                   // their tie keys 2 * p + bit (0x7fffffff: not a child)
    __shared__ double lam_lds[LMAX];
    const int lane = threadIdx.x;
    for (int i = lane; i < PSCL_EXP_TABLE_WORDS; i += 64) T[i] = P.exp_table[i];
    __syncthreads();

    const int N = P.N, n = P.n, K = P.K, L = P.L, W = P.W, NW = N >> 6;
    const bool path_lane = lane < LMAX;
    const int cpath = lane & (LMAX - 1);
    unsigned char* base = reinterpret_cast<unsigned char*>(P.long_scratch) + (size_t)blockIdx.x * P.long_block_bytes;
    double* tree = reinterpret_cast<double*>(base);
    uint64_t* ubuf = reinterpret_cast<uint64_t*>(base + long_tree_doubles(N, LMAX) * 8);  // [2][LMAX][NW]
    double* hist_llr = reinterpret_cast<double*>(ubuf + 2 * LMAX * NW);                  // [K][L]
    uint8_t* hist_par = reinterpret_cast<uint8_t*>(hist_llr + (HIST ? (size_t)K * L : 0));  // [N][L]
    auto info_bit = [&](int phi) { return (bool)((P.info_words[phi >> 6] >> (phi & 63)) & 1ULL); };

    const int64_t Bn = P.d_count ? (*P.d_count < P.B ? (int64_t)*P.d_count : P.B) : P.B;
    for (int64_t f = blockIdx.x; f < Bn; f += gridDim.x) {
        const int64_t frow = P.fidx ? P.fidx[f] : f;
        const int64_t fo = P.out_by_row ? frow : f;  // output row (the re-decode of screened frames: their own rows)
        // depth 0: the channel row (NR: de-rate-match + de-interleave while staging)
        if (P.rm_E == 0) {
            const double* src = P.llr + frow * N;
            for (int x = lane; x < N; x += 64) tree[x] = src[x];
        } else {
            const double* src = P.llr + frow * P.rm_E;
            for (int x = lane; x < N; x += 64) tree[x] = nr_stage(src, P.rm_src[x], P.rm_E, N);
        }
        for (int x = lane; x < NW; x += 64) ubuf[x] = 0;  // path 0's bits, buffer 0
        wave_mem_fence();
        const uint64_t* fr = P.force ? P.force + f * 2 * W : nullptr;

        double metric = 0.0;
        uint64_t tab = 0;     // slot of each depth 1..n-1 (5 bits per depth)
        uint32_t lastbit = 0;
        int cnt = 1, j = 0, cur = 0;

        for (int phi = 0; phi < N; ++phi) {
            const int t = phi ? __builtin_ctz((unsigned)phi) : n;
            const int start = phi ? n - t : 1;
            const int w = N >> start;  // width of the g node's left sibling (= 2^t)
            uint64_t xs = 0;           // its partial sums, w <= 64 (path lanes)
            const uint64_t* ucur = ubuf + (size_t)cur * LMAX * NW;
            if (phi && start <= n - 1) {
                if (w <= 64) {
                    if (lane < cnt) {
                        const int lo = phi - w;
                        const uint64_t word = ucur[(size_t)lane * NW + (lo >> 6)];
                        xs = polar_transform64(w == 64 ? word : (word >> (lo & 63)) & ((1ULL << w) - 1));
                    }
                } else {
                    const int nwd = w >> 6, w0 = (phi - w) >> 6;
                    for (int it = lane; it < cnt * nwd; it += 64)
                        xsw[(it / nwd) * kMaxXsWords + it % nwd] = polar_transform64(ucur[(size_t)(it / nwd) * NW + w0 + it % nwd]);
                    wave_lds_fence();
                    for (int s = 1; s < nwd; s <<= 1) {  // cross-word stages: word k ^= word k + s, (k & s) == 0
                        for (int it = lane; it < cnt * nwd; it += 64) {
                            const int p = it / nwd, k = it % nwd;
                            if (!(k & s)) xsw[p * kMaxXsWords + k] ^= xsw[p * kMaxXsWords + k + s];
                        }
                        wave_lds_fence();
                    }
                }
            }
            // ---- tree: depths start .. n-1 of every live path
            if (start <= n - 1) {
                if (path_lane) {
                    tab_lds[lane] = tab;
                    xs_lds[lane] = xs;
                }
                wave_lds_fence();
            }
            for (int d = start; d <= n - 1; ++d) {
                const int wd = N >> d;
                const bool is_g = d == start && phi;
                const bool first = d == start;  // (wave-uniform)
                for (int it = lane; it < cnt * wd; it += 64) {
                    const int p = it / wd, e = it % wd;
                    const int ps = first ? (d == 1 ? 0 : long_slot(tab_lds[p], d - 1)) : p;
                    const double* par = d == 1 ? tree : tree + long_node_off(N, LMAX, d - 1, ps);
                    const double a = par[e], b = par[e + wd];
                    double v;
                    if (is_g) {
                        const uint32_t bit = w <= 64 ? (uint32_t)(xs_lds[p] >> e) & 1u
                                                     : (uint32_t)(xsw[p * kMaxXsWords + (e >> 6)] >> (e & 63)) & 1u;
                        v = g_node(a, b, bit);
                    } else {
                        v = f_minsum(a, b);
                    }
                    tree[long_node_off(N, LMAX, d, p) + e] = v;
                }
                wave_mem_fence();
            }
            if (start <= n - 1) {  // own slot at every rewritten depth
                for (int d = start; d <= n - 1; ++d)
                    tab = (tab & ~(31ULL << (5 * (d - 1)))) | ((uint64_t)cpath << (5 * (d - 1)));
            }
            // ---- leaf LLR (path lanes)
            double lam = 0.0;
            if (path_lane && lane < cnt) {
                const double* par = n == 1 ? tree : tree + long_node_off(N, LMAX, n - 1, start <= n - 1 ? lane : long_slot(tab, n - 1));
                lam = (phi & 1) ? g_node(par[0], par[1], lastbit) : f_minsum(par[0], par[1]);
            }
            // ---- children metrics (scl.py:102-105): path lane p publishes the keys of its two
            // children, candidate p (bit 0) and candidate p + LMAX (bit 1), with the state the
            // survivors inherit.  (The exchange goes through LDS: this kernel is not the hot
            // path, and plain LDS traffic keeps it clear of cross-lane hazards.)
            const bool is_info = info_bit(phi);
            int ncnt = cnt;
            if (is_info && !P.sc_hard && !(fr && ((fr[j >> 6] >> (j & 63)) & 1))) ncnt = 2 * cnt < L ? 2 * cnt : L;
            if (path_lane) {
                const double Lt = pscl_softplus_tail_bf(lam, T);
                const double m0 = metric + pscl_logaddexp0(-lam, Lt), m1 = metric + pscl_logaddexp0(lam, Lt);
                bool v0 = lane < cnt, v1 = lane < cnt;
                if (!is_info) {
                    v1 = false;  // frozen: bit 0 (scl.py:149-153)
                } else if (P.sc_hard) {
                    const bool one = lam < 0.0;  // sc_decode (polar.py:149-153)
                    v0 = v0 && !one;
                    v1 = v1 && one;
                } else if (fr && ((fr[j >> 6] >> (j & 63)) & 1)) {
                    const bool one = (fr[W + (j >> 6)] >> (j & 63)) & 1;  // forced (scl.py:146-161)
                    v0 = v0 && !one;
                    v1 = v1 && one;
                }
                key_lds[lane] = v0 ? pscl_asu64(m0) : 0x7ff0000000000000ULL;  // +inf: behind every live child
                key_lds[lane + LMAX] = v1 ? pscl_asu64(m1) : 0x7ff0000000000000ULL;
                kt_lds[lane] = v0 ? 2u * (uint32_t)lane : 0x7fffffffu;
                kt_lds[lane + LMAX] = v1 ? 2u * (uint32_t)lane + 1u : 0x7fffffffu;
                tab_lds[lane] = tab;
                lam_lds[lane] = lam;
            }
            wave_lds_fence();
            // stable rank (scl.py:173-174): keys (metric, 2 * list position + bit) smaller than
            // mine; metrics are >= 0, so their bit patterns order as the values do
            uint32_t r = 0;
            bool kval = false;
            if (lane < G) {
                const uint64_t km = key_lds[lane];
                const uint32_t kt = kt_lds[lane];
                kval = kt != 0x7fffffffu;
                for (int i = 0; i < G; ++i) {
                    const uint64_t ki = key_lds[i];
                    r += (ki < km || (ki == km && kt_lds[i] < kt)) ? 1u : 0u;
                }
            }
            if (kval && r < (uint32_t)ncnt) inv[r] = (uint8_t)lane;
            wave_lds_fence();
            const int c = lane < ncnt ? inv[lane] : (lane & (G - 1));
            const int par_p = c & (LMAX - 1);
            const uint32_t b = c >= LMAX ? 1u : 0u;
            const uint64_t nm = key_lds[c];
            const uint64_t ntab = tab_lds[par_p];
            const double nlam = HIST ? lam_lds[par_p] : 0.0;
#ifdef PSCL_DEBUG_LONG
            if (f == 0 && phi < PSCL_DEBUG_LONG && lane < G)
                printf("phi %d info %d lane %d lam %.6f r %u c %d nm %016llx\n", phi, (int)is_info, lane, lam, r, c,
                       (unsigned long long)nm);
#endif
            // survivors' bits: copy the parent's words (up to word phi/64) and set bit phi
            uint64_t* unext = ubuf + (size_t)(cur ^ 1) * LMAX * NW;
            const int nw_used = (phi >> 6) + 1;
            for (int it = lane; it < ncnt * nw_used; it += 64) {
                const int q = it / nw_used, k = it % nw_used;
                const int cq = inv[q];
                uint64_t word = ucur[(size_t)(cq & (LMAX - 1)) * NW + k];
                if (k == (phi >> 6)) {  // bits of phases < phi only (the word's upper bits were never written)
                    word &= (1ULL << (phi & 63)) - 1;
                    if (cq >= LMAX) word |= 1ULL << (phi & 63);
                }
                unext[(size_t)q * NW + k] = word;
            }
            if (HIST && path_lane && lane < ncnt) {
                if (is_info) hist_llr[(size_t)j * L + lane] = nlam;  // decision LLR (scl.py:158,166)
                hist_par[(size_t)phi * L + lane] = (uint8_t)par_p;    // list position before this phase
            }
            wave_mem_fence();  // inv[] and the bit buffers are rewritten next phase
            metric = pscl_asf64(nm);
            tab = ntab;
            lastbit = b;
            cnt = ncnt;
            cur ^= 1;
            if (is_info) ++j;
        }

        // ---- epilogue: candidates u[info_set], CRC syndrome, best = first CRC pass (scl.py:176-209)
        const uint64_t* ufin = ubuf + (size_t)cur * LMAX * NW;
        const bool active = path_lane && lane < cnt;
        uint32_t syn = 0;
        if (active && P.has_crc)
            for (int jj = 0; jj < K; ++jj) {
                const int ph = P.info_set[jj];
                if ((ufin[(size_t)lane * NW + (ph >> 6)] >> (ph & 63)) & 1ULL) syn ^= P.crc_cols[jj];
            }
        const uint64_t passmask = __ballot(active && syn == 0);
        const int best = (P.has_crc && passmask) ? __builtin_ctzll(passmask) : 0;
        auto cand_word = [&](int q, int wi) {  // candidate bits 64*wi .. of path q
            uint64_t word = 0;
            for (int jj = 64 * wi; jj < K && jj < 64 * wi + 64; ++jj) {
                const int ph = P.info_set[jj];
                word |= ((ufin[(size_t)q * NW + (ph >> 6)] >> (ph & 63)) & 1ULL) << (jj & 63);
            }
            return word;
        };
        if (active) {
            const int64_t row = fo * L + lane;
            if (P.metrics) P.metrics[row] = metric;
            if (P.cands)
                for (int wi = 0; wi < W; ++wi) P.cands[row * W + wi] = cand_word(lane, wi);
            if (HIST && P.info_llrs) {  // trace the path back through every phase
                int cur_q = lane, jj = K - 1;
                for (int ph = N - 1; ph >= 0; --ph) {
                    if (info_bit(ph)) {
                        P.info_llrs[row * K + jj] = hist_llr[(size_t)jj * L + cur_q];
                        --jj;
                    }
                    cur_q = hist_par[(size_t)ph * L + cur_q];
                }
            }
            if (lane == best) {
                const bool bpass = P.has_crc ? (syn == 0) : true;
                if (HIST && P.best_info_llrs) {
                    int cur_q = lane, jj = K - 1;
                    for (int ph = N - 1; ph >= 0; --ph) {
                        if (info_bit(ph)) {
                            P.best_info_llrs[fo * K + jj] = hist_llr[(size_t)jj * L + cur_q];
                            --jj;
                        }
                        cur_q = hist_par[(size_t)ph * L + cur_q];
                    }
                }
                int bit_err = 0, pay_err = 0;
                for (int wi = 0; wi < W; ++wi) {
                    const uint64_t word = cand_word(lane, wi);
                    if (P.best) P.best[fo * W + wi] = word;
                    if (P.ref) {
                        const uint64_t dff = word ^ P.ref[fo * W + wi];
                        const int kp = P.k_payload - 64 * wi;
                        const uint64_t pm = kp >= 64 ? ~0ULL : (kp > 0 ? ((1ULL << kp) - 1) : 0ULL);
                        bit_err += __popcll(dff);
                        pay_err += __popcll(dff & pm);
                    }
                }
                if (P.flags) P.flags[fo] = (uint8_t)((bpass ? PSCL_FLAG_CRC_PASS : 0u) | (uint32_t)best);
                if (P.n_paths) P.n_paths[fo] = cnt;
                if (P.ref) {  // run_fer_sweep.py:91-109, run_ber_sweep.py:77-82,156
                    unsigned long long* C = reinterpret_cast<unsigned long long*>(P.counters);
                    if (!bpass) atomicAdd(C + PSCL_CNT_FRAME_ERR, 1ULL);
                    if (bit_err) atomicAdd(C + PSCL_CNT_BIT_ERR, (unsigned long long)bit_err);
                    if (pay_err) {
                        atomicAdd(C + PSCL_CNT_PAYLOAD_ERR, 1ULL);
                        atomicAdd(C + PSCL_CNT_PAYLOAD_BIT, (unsigned long long)pay_err);
                    }
                }
            }
        }
        wave_mem_fence();  // the next frame reuses this workgroup's scratch
    }
    if (P.ref && !P.out_by_row && blockIdx.x == 0 && threadIdx.x == 0)
        atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + PSCL_CNT_FRAMES, (unsigned long long)P.B);
}

template <int LMAX>
hipError_t launch_long_l(const pscl_decode_params& P, int hist, int64_t grid, hipStream_t s) {
    if (hist)
        hipLaunchKernelGGL((scl_long_kernel<LMAX, true>), dim3((unsigned)grid), dim3(64), 0, s, P);
    else
        hipLaunchKernelGGL((scl_long_kernel<LMAX, false>), dim3((unsigned)grid), dim3(64), 0, s, P);
    return hipGetLastError();
}

}  // namespace

int64_t pscl_long_block_bytes(int N, int L, int K, int hist) {
    const int lmax = pscl_decode_lmax(L);
    int64_t b = long_tree_doubles(N, lmax) * 8 + (int64_t)2 * lmax * (N / 64) * 8;
    if (hist) b += (int64_t)K * L * 8 + (int64_t)N * L;
    return (b + 255) & ~(int64_t)255;
}

// resident one-wave workgroups per CU for list size bucket LMAX (the smaller of the plain and
// history instances: one grid size serves both); 16 when the runtime cannot tell (no device)
template <int LMAX>
static int long_blocks_per_cu() {
    int a = 0, b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, reinterpret_cast<const void*>(scl_long_kernel<LMAX, false>), 64, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, reinterpret_cast<const void*>(scl_long_kernel<LMAX, true>), 64, 0) != hipSuccess)
        return 16;
    const int m = a < b ? a : b;
    return m < 1 ? 1 : (m > 32 ? 32 : m);
}

int64_t pscl_long_grid(int64_t B, int L) {
    // one wavefront per frame is latency-bound: fill every resident wave slot (64 VGPRs per
    // lane: 8 waves per SIMD), each wave striding over frames
    static int cus = 0, per_cu[6] = {0, 0, 0, 0, 0, 0};
    if (!cus) {
        int dev = 0, n = 0;
        cus = (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
                  ? n
                  : 256;
    }
    const int lmax = pscl_decode_lmax(L), li = __builtin_ctz((unsigned)lmax);
    if (!per_cu[li]) {
        switch (lmax) {
            case 1: per_cu[li] = long_blocks_per_cu<1>(); break;
            case 2: per_cu[li] = long_blocks_per_cu<2>(); break;
            case 4: per_cu[li] = long_blocks_per_cu<4>(); break;
            case 8: per_cu[li] = long_blocks_per_cu<8>(); break;
            case 16: per_cu[li] = long_blocks_per_cu<16>(); break;
            default: per_cu[li] = long_blocks_per_cu<32>(); break;
        }
    }
    const int64_t cap = (int64_t)cus * per_cu[li];
    return B < 1 ? 1 : (B < cap ? B : cap);
}

hipError_t pscl_launch_long(const pscl_decode_params& P, int hist, hipStream_t s) {
    if (P.N > kMaxLongN || P.N < 256 || !P.long_scratch || !P.info_words) return hipErrorInvalidValue;
    const int64_t grid = pscl_decode_grid(P);
    switch (pscl_decode_lmax(P.L)) {
        case 1: return launch_long_l<1>(P, hist, grid, s);
        case 2: return launch_long_l<2>(P, hist, grid, s);
        case 4: return launch_long_l<4>(P, hist, grid, s);
        case 8: return launch_long_l<8>(P, hist, grid, s);
        case 16: return launch_long_l<16>(P, hist, grid, s);
        default: return launch_long_l<32>(P, hist, grid, s);
    }
}
