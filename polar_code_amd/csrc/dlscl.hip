// dlscl.hip -- DL-SCL bit-flip retry rounds on the device (dlscl/flip.py:65-141).
//
// The retry loop of decode_with_retries runs over a compacted list of the frames whose
// baseline SCL best candidate fails the CRC.  Each frame keeps, in an "entry" slot, the
// state the reference threads through its loop (flip.py:110-136): the set of tried indices
// and the latest attempt's best bits (the reference bits of the next force vector).  A round
// is two launches:
//   decode            the SCL kernel on the round's entries (LLR row by indirection, forced
//                     bits), warm-started past each entry's forced prefix (below)
//   dl_post_kernel    per entry: replay of the attempt's best path (all leaf LLRs, hence L0,
//                     flip.py:127-132), final-attempt bookkeeping and the CRC stop rule
//                     (flip.py:123-136); for the survivors the next flip -- q = |L0| @ beta,
//                     argmin over untried (q, index) (flip.py:104-111) -- its force vector
//                     (flip.py:30-34) and the warm-start state of its forced prefix
// A first post pass over the baseline results (init) selects every entry's first flip.
// Frames never leave the GPU; the live counts stay on the device.
//
// Warm start.  A retry forces the reference bits on info indices [0, idx) and the flipped bit
// at idx: up to the flipped phase phi* = info_set[idx] the list holds ONE path whose bits are
// known, so its leaf LLRs are the replayed ones and its metric is their exact increments summed
// in phase order.  The post pass writes that metric at every 16-phase boundary below phi*
// (warm_metric[e][k], k <= phi* / 16) and appends the entry to bucket phi* / 16 of the next
// round's list; the decode kernel maps its frames to entries bucket by bucket and starts each
// wavefront at phase 16 k of its first frame's bucket (scl128_impl.h), skipping 16 k phases of
// tree walk, metric tails and list updates per frame -- half the phases on average at 5 dB.
//
// Why a replay instead of the decoder's history: the decision LLR of a path at info phase
// j (scl.py:158,166) is a function of the channel LLRs and the path's own earlier bits only
// (lazy copies share, never alter, ancestors' values).  With the final bits known, every
// leaf LLR follows top-down, level by level, through the same f/g operations -- bit-identical
// values at ~1/15 of a decode, and the decode itself keeps the occupancy of the plain kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "polar_scl.h"
#include "scl_device.h"
#include "scl_kernels.h"

#pragma clang fp contract(off)

namespace {

using pscl::f_minsum;
using pscl::g_node;
using pscl::polar_transform64;

// cross-lane steps of the post pass's per-entry reductions: DPP within a 16-lane row (quad_perm xor 1,
// xor 2, the half-row mirror i <-> 7 - i, the row mirror i <-> 15 - i: after the four every lane
// holds its row's reduction), then one swizzle-free exchange between the two rows of a 32-lane entry
// -- VALU-latency steps where ds_bpermute round trips had been
template <int CTRL>
__device__ __forceinline__ uint32_t post_dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ uint64_t post_dpp64(uint64_t v) {
    return ((uint64_t)post_dpp32<CTRL>((uint32_t)(v >> 32)) << 32) | post_dpp32<CTRL>((uint32_t)v);
}
// (steps: quad_perm [1,0,3,2] = 0xB1, [2,3,0,1] = 0x4E, row_half_mirror 0x141, row_mirror 0x140)

// the value of lane (lane ^ W) within a 32-lane entry half (W = 1..16): quad_perm xor 1 / xor 2,
// xor 4 as the half-row mirror then quad_perm xor 3, xor 8 as row_ror:8, xor 16 across the two rows
template <int W>
__device__ __forceinline__ uint64_t post_xor64(uint64_t v, int lane) {
    if constexpr (W == 1) return post_dpp64<0xB1>(v);
    else if constexpr (W == 2) return post_dpp64<0x4E>(v);
    else if constexpr (W == 4) return post_dpp64<0x1B>(post_dpp64<0x141>(v));
    else if constexpr (W == 8) return post_dpp64<0x128>(v);
    else return pscl::shfl_u64(v, lane ^ 16);
}

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
        if (list) list[pos] = pos;
    }
}

__global__ void __launch_bounds__(256) iota64_kernel(int64_t* out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = i;
}

// Channel LLRs p = lane and lane + 64 of a frame row (rate matched: de-rate-matched and
// de-interleaved on the fly); N <= 128
__device__ __forceinline__ void load_row(const double* llr_row, int rm_E, const int32_t* rm_src, int N, double& c0,
                                         double& c1) {
    const int lane = threadIdx.x & 63;
    c0 = c1 = 0.0;
    if (lane < N) c0 = rm_E == 0 ? llr_row[lane] : pscl::nr_stage(llr_row, rm_src[lane], rm_E, N);
    if (lane + 64 < N) c1 = rm_E == 0 ? llr_row[lane + 64] : pscl::nr_stage(llr_row, rm_src[lane + 64], rm_E, N);
}

// Leaf LLRs of a path with information bits (b0, b1), top-down through the tree (one
// wavefront; channel values c0, c1 from load_row; cur, nxt: 128-double LDS buffers).  Returns
// the buffer holding the N leaves; u[h] = the path's bits u[64 h + lane] (ballots), jpos[h] =
// info index of phase 64 h + lane (or -1).
__device__ __forceinline__ double* replay_leaves(double c0, double c1, int N, int n, const uint64_t* info_mask,
                                                 uint64_t b0, uint64_t b1, double* cur, double* nxt, uint64_t* u,
                                                 int* jpos) {
    const int lane = threadIdx.x & 63;
    if (lane < N) cur[lane] = c0;
    if (lane + 64 < N) cur[lane + 64] = c1;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int p = lane + 64 * h;
        bool bit = false;
        jpos[h] = -1;
        if (p < N && ((info_mask[h] >> lane) & 1ULL)) {
            const int j = (h ? __popcll(info_mask[0]) : 0) + __popcll(info_mask[h] & ((1ULL << lane) - 1ULL));
            jpos[h] = j;
            bit = ((j < 64 ? b0 : b1) >> (j & 63)) & 1ULL;
        }
        u[h] = __ballot(bit);
    }
    pscl::wave_lds_fence();
    // Partial sums: the g node k2 (odd) of width w = 2^m takes bit i of the transform of
    // u[(k2-1) w, k2 w), which is bit (k2-1) w + i of X_m = u after butterfly stages 1, 2, ..,
    // 2^(m-1) (polar_transform64 stage by stage: the later stages do not mix an aligned w-bit
    // segment).  The stages are involutions that commute, so X_{m-1} = stage 2^(m-1) of X_m:
    // one wave-uniform (scalar) stage per level instead of a full transform per element.
    auto stage = [](uint64_t x, int s) {
        const uint64_t M = s == 1 ? 0x5555555555555555ULL : s == 2 ? 0x3333333333333333ULL
                         : s == 4 ? 0x0f0f0f0f0f0f0f0fULL : s == 8 ? 0x00ff00ff00ff00ffULL
                         : s == 16 ? 0x0000ffff0000ffffULL : 0x00000000ffffffffULL;
        return x ^ ((x >> s) & M);
    };
    uint64_t X0 = u[0], X1 = u[1];
    for (int m = 1; m < n; ++m) {  // X_{n-1}
        X0 = stage(X0, 1 << (m - 1));
        X1 = stage(X1, 1 << (m - 1));
    }
    for (int d = 0; d < n; ++d) {
        const int lw2 = n - d - 1, w2 = 1 << lw2;
        for (int p2 = lane; p2 < N; p2 += 64) {
            const int k2 = p2 >> lw2, i = p2 & (w2 - 1);
            const int pa = ((k2 >> 1) << (lw2 + 1)) + i;
            const double a = cur[pa], bb = cur[pa + w2];
            double v;
            if (!(k2 & 1)) {
                v = f_minsum(a, bb);
            } else {
                const int q = p2 - w2;  // bit (k2-1) w2 + i of X_lw2
                v = g_node(a, bb, (uint32_t)(((q >> 6) ? X1 : X0) >> (q & 63)) & 1u);
            }
            nxt[p2] = v;
        }
        pscl::wave_lds_fence();
        double* t = cur;
        cur = nxt;
        nxt = t;
        if (lw2 > 0) {
            X0 = stage(X0, w2 >> 1);
            X1 = stage(X1, w2 >> 1);
        }
    }
    return cur;
}

// one wavefront per entry: leaf LLRs of the entry's path (bits given), written at its info
// positions.  LDS: two 128-double level buffers per wave.
__global__ void __launch_bounds__(256) replay_kernel(const pscl_replay_params R, int64_t cap) {
    __shared__ double lvl[4][2][PSCL_FAST_N];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + wave;
    if (b >= *R.count || b >= cap) return;
    const int e = R.list ? R.list[b] : (int)b;
    const int64_t row = R.act[e];
    const uint64_t* bw = R.bits + (R.bits_by_row ? row : b) * R.W;
    uint64_t u[2];
    int jpos[2];
    double c0, c1;
    load_row(R.llr + row * (R.rm_E ? R.rm_E : R.N), R.rm_E, R.rm_src, R.N, c0, c1);
    const double* cur = replay_leaves(c0, c1, R.N, R.n, R.info_mask, bw[0], R.W > 1 ? bw[1] : 0ULL, lvl[wave][0],
                                      lvl[wave][1], u, jpos);
    double* out = R.out + (int64_t)e * R.K;
#pragma unroll
    for (int h = 0; h < 2; ++h)
        if (jpos[h] >= 0) out[jpos[h]] = cur[lane + 64 * h];
}

// Timing-only ablations of dl_post_kernel (tools/build_variant.py --unit dlscl
// -DPSCL_POST_ABLATE=m; 0 in the product, results invalid otherwise): 1 no bucket atomics,
// 2 no warm-start tails, 4 no flip metric (q = |L0|), 8 no serial prefix sums, 64 no exact
// fallback of uncertified packed flip sums
#ifndef PSCL_POST_ABLATE
#define PSCL_POST_ABLATE 0
#endif

// One post pass of the retry loop (see the header).  Each wavefront works on two entries at
// a time, one per 32-lane half (4 tree elements and up to 4 flip candidates per lane), so a
// workgroup keeps twice the entries in flight that one entry per wavefront allowed (the pass
// is latency-bound: LDS round trips of the replay levels, the flip metric's sums, the serial
// prefix sums).  Workgroups of 4 wavefronts own contiguous ranges of the pass's entries; every
// wavefront preloads the metadata of its next 64 entries (one lane each: entry id, frame,
// bits, flags, tried state) and prefetches the next pair's channel rows while it replays the
// current pair.  Survivors are staged in LDS and appended to the next round's bucket lists
// with one global atomic per (workgroup, bucket) per 512 entries: one atomic per entry put
// ~5k same-address device atomics on each bucket counter (measured: 316 of 467 us of the
// first pass at L = 4, 5 dB).  The exp table of the exact metric tails is staged in LDS once
// per workgroup, and beta (when K * K doubles fit) too.  Pipelined DL-SCL calls
// (pscl_set_pipelined, Q.narrow) take a narrow form instead: workgroups of 4 wavefronts with beta
// read through L2 (~20 KB of LDS against ~70 KB), which fit beside the next call's baseline decode
// running concurrently -- a post pass that needs 70 KB of free LDS on one CU waits for that
// baseline to end (measured, config 4 pipelined: 3.86-3.93 -> 3.54-3.58 ms per step; 8
// wavefronts with beta through L2 4.10, 4 with beta staged 3.91).  Alone on the GPU the wide
// form is the faster one (the FER sweep's 4.0 dB point: 16.6 against 34 ms).
#ifndef PSCL_POST_GRID
#define PSCL_POST_GRID 512
#endif
#ifndef PSCL_POST_PAIRS
#define PSCL_POST_PAIRS 2
#endif
// unroll of the flip metric's sums over k: beta rows in flight per lane (read through L2 in the
// narrow form)
// occupancy hint of the post pass (waves per SIMD): 3 (168 VGPRs) -- at 4 (128 VGPRs) it spilled
// 5 VGPRs to scratch (24 B per lane), and a kernel with scratch stalls its first dispatch on each
// queue while the runtime allocates that queue's scratch; a pass's grid (512 workgroups of 4 or 8
// wavefronts) is resident either way
#ifndef PSCL_POST_WPE
#define PSCL_POST_WPE 3
#endif
#ifndef PSCL_POST_UNROLL
#define PSCL_POST_UNROLL 4
#endif
#ifndef PSCL_POST_BETA32
#define PSCL_POST_BETA32 1
#endif
#ifndef PSCL_POST_BETA_LDS
#define PSCL_POST_BETA_LDS 1
#endif
// the flip metric's sums with fused multiply-adds, certified against the exact sums' bound (1), or
// the exact index-order sums throughout (0)
// the packed fp32 flip sums of the 2-entry narrow form on the matrix cores (1: v_mfma_f32_16x16x4_f32,
// bit for bit the same k-ordered fp32 fma chains, MI355X_MICROARCH.md, leaving the VALU to the decode
// beside it), or as v_pk_fma_f32 on the VALU (0).  Measured (profiles/r06v_post_mfma_ab.txt): bit-
// identical, config 4 2.27 against 2.19 ms -- a post wavefront's 64 MFMAs (16 columns, 2 used) hold
// its slot and LDS ~2,000 cycles longer per entry pair, and that costs the decode more than the
// VALU cycles it gives back: off
#ifndef PSCL_POST_MFMA
#define PSCL_POST_MFMA 0
#endif
#ifndef PSCL_POST_FMA
#define PSCL_POST_FMA 1
#endif
#ifndef PSCL_POST_WAVES_NARROW
#define PSCL_POST_WAVES_NARROW 4
#endif
constexpr int kPostWavesWide = 8, kPostWavesNarrow = PSCL_POST_WAVES_NARROW;
// entries per wavefront at a time (dl_post_kernel EPW): the narrow form (pipelined calls, beside the
// next baseline: its cost is the wave slots it holds) and the wide one (a chain alone: latency)
#ifndef PSCL_POST_EPW_NARROW
#define PSCL_POST_EPW_NARROW 2  // (K = 64; PSCL_TUNE_POST_EPW)
#endif
#ifndef PSCL_POST_WPE_Q  // (occupancy hint of the 4-entry form)
#define PSCL_POST_WPE_Q 3
#endif
#ifndef PSCL_POST_EPW_WIDE
#define PSCL_POST_EPW_WIDE 2
#endif
constexpr int kPostEpwNarrow = PSCL_POST_EPW_NARROW, kPostEpwWide = PSCL_POST_EPW_WIDE;
constexpr int kPostIters = 32;  // entry pairs per wavefront between flushes

template <int PW, int EPW>
struct PostShared {
    static constexpr int kChunk = PW * 2 * kPostIters;  // entries per workgroup between flushes (64 per wavefront)
    double lvl[PW][EPW][2][PSCL_FAST_N];  // [wave][entry slot][buffer][element]
    uint64_t exp_table[PSCL_EXP_TABLE_WORDS];
    int32_t st_e[kChunk];
    uint16_t st_pos[kChunk];
    uint8_t st_seg[kChunk];
    int32_t lcnt[PSCL_DL_NSEG];
    int32_t gbase[PSCL_DL_NSEG];
    int32_t nst;
};

// Channel LLRs p = hl + HLN m (m < 128 / HLN) of a frame row, N <= 128 (HLN lanes per entry)
template <int HLN>
__device__ __forceinline__ void load_rowq(const double* row, int rm_E, const int32_t* rm_src, int N, int hl, double* c) {
#pragma unroll
    for (int m = 0; m < PSCL_FAST_N / HLN; ++m) {
        const int p = hl + HLN * m;
        c[m] = p < N ? (rm_E == 0 ? row[p] : pscl::nr_stage(row, rm_src[p], rm_E, N)) : 0.0;
    }
}

// per-entry broadcast of lane base + hs's value to entry slot hs (base wave-uniform): one scalar read
// per slot and a select, not a ds_bpermute round trip
template <int EPW>
__device__ __forceinline__ uint32_t slot_bcast32(uint32_t v, int base, int hs) {
    uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)v, base);
#pragma unroll
    for (int k = 1; k < EPW; ++k) {
        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)v, base + k);
        r = hs == k ? x : r;
    }
    return r;
}
template <int EPW>
__device__ __forceinline__ uint64_t slot_bcast64(uint64_t v, int base, int hs) {
    return ((uint64_t)slot_bcast32<EPW>((uint32_t)(v >> 32), base, hs) << 32) | slot_bcast32<EPW>((uint32_t)v, base, hs);
}

// NC, KC: N and K compiled in (128 and 64 / 88: the BASELINE codes) or 0 (from Q).  EPW: entries a
// wavefront works on at a time, HLN = 64 / EPW lanes each (2: halves of 32 lanes, 4 elements and 2
// candidates per lane; 4: quarters of 16 lanes, 8 elements and 4 candidates per lane -- the same
// instructions per entry, twice the entries per wavefront latency)
template <int NC, int KC, int PW, int EPW = 2>
__global__ void __launch_bounds__(PW * 64) __attribute__((amdgpu_waves_per_eu(EPW == 4 ? PSCL_POST_WPE_Q : PSCL_POST_WPE))) dl_post_kernel(const pscl_post_params Q, int beta_lds) {
    static_assert(EPW == 2 || EPW == 4, "entries per wavefront");
    constexpr int kPostWaves = PW, kPostChunk = PostShared<PW, EPW>::kChunk;
    constexpr int HLN = 64 / EPW, EL = PSCL_FAST_N / HLN;  // lanes per entry, tree elements per lane
    constexpr bool K1 = KC > 0 && KC <= 64;                 // one word of information bits
    // (sums unrolled less in the 4-entry form: its twice as many candidates per lane hold the loads)
    constexpr int kSumUnroll = EPW == 4 ? 2 : PSCL_POST_UNROLL, kPkUnroll = EPW == 4 ? 2 : 4;
    constexpr bool MF = PSCL_POST_MFMA && KC == 64 && EPW == 2;  // (flip sums on the matrix cores)
    __shared__ PostShared<PW, EPW> S;
    extern __shared__ double sbeta[];  // [K][K]: fp64 when beta_lds == 1, fp32 when 2
    float* const sbeta32 = reinterpret_cast<float*>(sbeta);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int hs = lane / HLN, hl = lane % HLN, hb = lane & ~(HLN - 1);  // entry slot, lane in slot, slot's first lane
    const int N = NC ? NC : Q.N, K = KC ? KC : Q.K, W = KC ? (KC + 63) / 64 : Q.W, n = NC ? 7 : Q.n;
    for (int i = threadIdx.x; i < PSCL_EXP_TABLE_WORDS; i += blockDim.x) S.exp_table[i] = Q.exp_table[i];
    if (beta_lds == 1)
        for (int i = threadIdx.x; i < K * K; i += blockDim.x) sbeta[i] = Q.beta[i];
    else if (beta_lds == 2) {
        if constexpr (MF) {  // [k][j ^ 16 (k & 3)]: the MFMA's A operand rows k = 4 s + kl, columns
                             // 16 t + jl read without bank conflicts (each kl group on its own 16 banks)
            for (int i = threadIdx.x; i < K * K; i += blockDim.x) {
                const int k = i >> 6, j = i & 63;
                sbeta32[k * 64 + (j ^ (16 * (k & 3)))] = (float)Q.beta[i];
            }
        } else if constexpr (KC == 64) {  // lane layout [k][hl][m] = beta[k][hl + HLN m]: one 8- (16-) byte
                                          // read gives a lane all of its 2 (4) candidates (the packed sums below)
            for (int i = threadIdx.x; i < K * K; i += blockDim.x) {
                const int k = i >> 6, j = i & 63;
                sbeta32[(k * HLN + (j % HLN)) * (64 / HLN) + (j / HLN)] = (float)Q.beta[i];
            }
        } else {
            for (int i = threadIdx.x; i < K * K; i += blockDim.x) sbeta32[i] = (float)Q.beta[i];
        }
    }
    if (threadIdx.x < PSCL_DL_NSEG) S.lcnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) S.nst = 0;
    const double* beta = beta_lds == 1 ? sbeta : Q.beta;  // (the exact sums: fp64 beta)
    const uint64_t info0 = Q.info_mask[0], info1 = Q.info_mask[1];
    const int ninfo0 = __popcll(info0);
    // information bits in the 16-phase blocks 0..b (b < 7), for the flip's warm-start segment
    int icum[PSCL_DL_NSEG - 1];
    {
        int acc = 0;
#pragma unroll
        for (int b = 0; b < PSCL_DL_NSEG - 1; ++b) {
            acc += __popcll(((b < 4 ? info0 : info1) >> (16 * (b & 3))) & 0xffffULL);
            icum[b] = acc;
        }
    }
    int pre[PSCL_DL_NSEG + 1];
    int64_t n_in;
    if (Q.init) {
        n_in = Q.cap;  // the entries are act[0, cap)
    } else {
        n_in = pscl_bucket_prefix(Q.in_count, Q.cap, pre);
    }
    if (n_in > Q.cap) n_in = Q.cap;
    const int64_t per = (n_in + gridDim.x - 1) / gridDim.x;
    const int64_t i_begin = (int64_t)blockIdx.x * per;
    const int64_t i_end = i_begin + per < n_in ? i_begin + per : n_in;
    unsigned long long decodes = 0;
    double* buf0 = S.lvl[wave][hs][0];
    double* buf1 = S.lvl[wave][hs][1];
    // info index of each of the lane's tree positions p = hl + HLN m (-1: frozen or beyond N),
    // packed a byte each (0xff: -1) -- 2 registers for the 8 positions of the quarter layout
    uint32_t jpk[(EL + 3) / 4];
#pragma unroll
    for (int i = 0; i < (EL + 3) / 4; ++i) jpk[i] = 0xffffffffu;
#pragma unroll
    for (int m = 0; m < EL; ++m) {
        const int p = hl + HLN * m;
        const uint64_t w = p < 64 ? info0 : info1;
        const bool inf = p < N && ((w >> (p & 63)) & 1ULL);
        const int j = p < 64 ? __popcll(info0 & ((1ULL << p) - 1ULL))
                             : ninfo0 + __popcll(info1 & ((1ULL << (p - 64)) - 1ULL));
        if (inf) jpk[m >> 2] = (jpk[m >> 2] & ~(0xffu << (8 * (m & 3)))) | ((uint32_t)j << (8 * (m & 3)));
    }
    auto jpos = [&](int m) -> int {
        const uint32_t v = (jpk[m >> 2] >> (8 * (m & 3))) & 0xffu;
        return v == 0xffu ? -1 : (int)v;
    };
    __syncthreads();
    for (int64_t cbase = i_begin; cbase < i_end; cbase += kPostChunk) {  // workgroup-uniform
        // metadata of this wavefront's entries of the chunk, lane l = entry cbase + 8 l + wave;
        // half s takes lane 2 it + s at iteration it
        const int64_t mi = cbase + (int64_t)lane * kPostWaves + wave;
        const bool mvalid = mi < i_end;
        int me = 0, mnt = 0;
        int64_t mf = 0;
        uint64_t mb0 = 0, mb1 = 0, mt0 = 0, mt1 = 0;
        uint32_t mfl = 0;
        if (mvalid) {
            if (Q.init) {
                me = (int)mi;
            } else {
                const int k = pscl_bucket_of(mi, pre);
                me = Q.in_list[(int64_t)k * Q.cap + (mi - pre[k])];
            }
            mf = Q.act[me];
            const uint64_t* bw = Q.init ? Q.best + mf * W : Q.ob + (int64_t)me * W;
            mb0 = bw[0];
            mb1 = W > 1 ? bw[1] : 0ULL;
            if (!Q.init) {
                mfl = Q.of[me];
                mnt = Q.ntried[me];
                mt0 = Q.tried[2 * me];
                mt1 = K1 ? 0ULL : Q.tried[2 * me + 1];  // (K <= 64: the upper tried word stays 0)
            }
        }
        const int nval = (int)__builtin_amdgcn_readfirstlane((int)__popcll(__ballot(mvalid)));  // lanes 0..nval-1
        const int npair = (nval + EPW - 1) / EPW;
        // channel rows of the first entries; the next iteration's rows are loaded into c as soon as
        // the replay has copied c to LDS (one row's registers live, not two)
        double c[EL];
        auto bc32 = [&](uint32_t v, int base) { return slot_bcast32<EPW>(v, base, hs); };
        auto bc64 = [&](uint64_t v, int base) { return slot_bcast64<EPW>(v, base, hs); };
        load_rowq<HLN>(Q.llr + (int64_t)bc64((uint64_t)mf, 0) * (Q.rm_E ? Q.rm_E : N), Q.rm_E, Q.rm_src, N, hl, c);
        for (int it = 0; it < npair; ++it) {
            const int sb = EPW * it, src = sb + hs;  // this entry slot's metadata lane
            bool valid = src < nval;
            const int e = (int)bc32((uint32_t)me, sb);
            const int64_t f = (int64_t)bc64((uint64_t)mf, sb);
            const uint64_t b0 = bc64(mb0, sb), b1 = K1 ? 0ULL : bc64(mb1, sb);
            const int nt = Q.init ? 0 : (int)bc32((uint32_t)mnt, sb);
            auto prefetch = [&]() {  // (metadata lanes past nval hold entry 0's: a valid row)
                if (it + 1 < npair)
                    load_rowq<HLN>(Q.llr + (int64_t)bc64((uint64_t)mf, sb + EPW) * (Q.rm_E ? Q.rm_E : N),
                                   Q.rm_E, Q.rm_src, N, hl, c);
            };
            bool more;
            if (Q.init) {  // baseline failing by construction (dl_compact); nothing tried yet
                more = valid && Q.rounds > 0;
            } else {       // the attempt just decoded is the frame's latest (flip.py:123-136)
                const uint32_t fl = bc32(mfl, sb);
                // (deferred by the screening retry decode: its exact decode and post pass follow)
                if (fl == PSCL_DL_DEFERRED) valid = false;
                if (valid && hl == 0) {
                    Q.best[f * W] = b0;
                    if (W > 1) Q.best[f * W + 1] = b1;
                    Q.flags[f] = (uint8_t)fl;
                    if (Q.attempts) Q.attempts[f] = nt + 1;
                }
                if (valid && hl == 0) ++decodes;
                more = valid && !(fl & PSCL_FLAG_CRC_PASS) && nt < Q.rounds;
            }
            if (!__ballot(more)) prefetch();
            if (__ballot(more)) {  // (wave-uniform: every slot runs the steps below; a slot with
                                   // nothing to do computes on its own buffers and writes nothing)
                // ---- replay: the leaves of the attempt's best path, level by level
                uint64_t u0 = 0, u1 = 0;  // the path's bits u[0..63], u[64..127] (this entry's)
#pragma unroll
                for (int m = 0; m < EL; ++m) {
                    const int j = jpos(m);
                    const bool bit = j >= 0 && (((K1 || j < 64 ? b0 : b1) >> (j & 63)) & 1ULL);
                    const uint64_t bm = __ballot(bit) >> hb;
                    const uint64_t part = bm & (HLN == 64 ? ~0ULL : ((1ULL << HLN) - 1ULL));
                    const int pos = HLN * m;  // (bits hl + HLN m: positions pos .. pos + HLN - 1)
                    if (pos < 64) u0 |= part << pos;
                    else u1 |= part << (pos - 64);
                }
                double* cur = buf0;
                double* nxt = buf1;
                // partial sums of level lw2 from X_lw2 = u after butterfly stages 1..2^(lw2-1)
                // (see replay_leaves)
                auto stage = [](uint64_t x, int st) {
                    const uint64_t M = st == 1 ? 0x5555555555555555ULL : st == 2 ? 0x3333333333333333ULL
                                     : st == 4 ? 0x0f0f0f0f0f0f0f0fULL : st == 8 ? 0x00ff00ff00ff00ffULL
                                     : st == 16 ? 0x0000ffff0000ffffULL : 0x00000000ffffffffULL;
                    return x ^ ((x >> st) & M);
                };
                uint64_t X0 = u0, X1 = u1;
                for (int mm = 1; mm < n; ++mm) {
                    X0 = stage(X0, 1 << (mm - 1));
                    X1 = stage(X1, 1 << (mm - 1));
                }
                int d0 = 0;  // first level through LDS
                // RR (N = 128, 32-lane entries): the whole replay in the lane's registers -- levels
                // w = 64 and 32 pair its own four positions hl + 32 m, levels w = 16 .. 1 pair
                // position p with p ^ w in lane hl ^ w (post_xor64); the leaves stay in lv[]
                constexpr bool RR = NC == 128 && EPW == 2;
                double lv[EL];
                if constexpr (RR) {
                    auto xb = [&](int q) { return (uint32_t)(((q >> 6) ? X1 : X0) >> (q & 63)) & 1u; };
                    const double v0 = f_minsum(c[0], c[2]), v1 = f_minsum(c[1], c[3]);
                    const double v2 = g_node(c[0], c[2], xb(hl)), v3 = g_node(c[1], c[3], xb(hl + 32));
                    X0 = stage(X0, 32);
                    X1 = stage(X1, 32);
                    lv[0] = f_minsum(v0, v1);
                    lv[1] = g_node(v0, v1, xb(hl));
                    lv[2] = f_minsum(v2, v3);
                    lv[3] = g_node(v2, v3, xb(hl + 64));
                    X0 = stage(X0, 16);
                    X1 = stage(X1, 16);
                    auto level = [&](auto WC) {
                        constexpr int w = decltype(WC)::value;
                        const bool hi = (hl & w) != 0;  // (the pair's second position: g, else f)
#pragma unroll
                        for (int m = 0; m < EL; ++m) {
                            const double oth = pscl_asf64(post_xor64<w>(pscl_asu64(lv[m]), lane));
                            const double a = hi ? oth : lv[m], bb = hi ? lv[m] : oth;
                            const double gv = g_node(a, bb, xb((hl ^ w) + 32 * m)), fv = f_minsum(a, bb);
                            lv[m] = hi ? gv : fv;
                        }
                        if constexpr (w > 1) {
                            X0 = stage(X0, w >> 1);
                            X1 = stage(X1, w >> 1);
                        }
                    };
                    level(std::integral_constant<int, 16>{});
                    level(std::integral_constant<int, 8>{});
                    level(std::integral_constant<int, 4>{});
                    level(std::integral_constant<int, 2>{});
                    level(std::integral_constant<int, 1>{});
                    d0 = n;
                } else {
#pragma unroll
                    for (int m = 0; m < EL; ++m)
                        if (hl + HLN * m < N) cur[hl + HLN * m] = c[m];
                }
                prefetch();
                pscl::wave_lds_fence();
                for (int d = d0; d < n; ++d) {
                    const int lw2 = n - d - 1, w2 = 1 << lw2;
#pragma unroll
                    for (int m = 0; m < EL; ++m) {
                        const int p2 = hl + HLN * m;
                        if (p2 < N) {
                            const int k2 = p2 >> lw2, i = p2 & (w2 - 1);
                            const int pa = ((k2 >> 1) << (lw2 + 1)) + i;
                            const double a = cur[pa], bb = cur[pa + w2];
                            const int q = (p2 - w2) & 127;  // bit (k2-1) w2 + i of X_lw2 (odd k2)
                            const double gv = g_node(a, bb, (uint32_t)(((q >> 6) ? X1 : X0) >> (q & 63)) & 1u);
                            const double fv = f_minsum(a, bb);
                            const uint64_t msk = (k2 & 1) ? ~0ULL : 0ULL;
                            nxt[p2] = pscl_asf64((pscl_asu64(gv) & msk) | (pscl_asu64(fv) & ~msk));
                        }
                    }
                    pscl::wave_lds_fence();
                    double* t = cur;
                    cur = nxt;
                    nxt = t;
                    if (lw2 > 0) {
                        X0 = stage(X0, w2 >> 1);
                        X1 = stage(X1, w2 >> 1);
                    }
                }
                // ---- |L0| at the information phases (flip.py:97-102, 127-132), in nxt
                // (K = 64, narrow form: an fp32 copy too, in nxt's upper half -- free until the tails)
                float* const l32 = reinterpret_cast<float*>(nxt + 64);
#pragma unroll
                for (int m = 0; m < EL; ++m)
                    if (jpos(m) >= 0) {
                        const double leaf = RR ? lv[m] : cur[hl + HLN * m];
                        nxt[jpos(m)] = fabs(leaf);
                        if (KC == 64 && beta_lds == 2) l32[jpos(m)] = (float)fabs(leaf);
                    }
                pscl::wave_lds_fence();
                // ---- next flip: argmin over untried (q, index), q = |L0| @ beta summed in
                // index order (flip.py:104-108), q = |L0| without beta
                const uint64_t t0 = Q.init ? 0ULL : bc64(mt0, sb), t1 = Q.init || K1 ? 0ULL : bc64(mt1, sb);
                uint64_t bk = ~0ULL;
                int bj = 0x7fffffff;
                // candidates j = hl + HLN m; their sums advance together (one |L0_k| read serves
                // all, and the dependent adds of the chains interleave)
                constexpr int MC = KC ? (KC + HLN - 1) / HLN : PSCL_FAST_N / HLN;
                double qv[MC];
                auto argmin = [&]() {  // (key, index) over the untried candidates of this half
                    bk = ~0ULL;
                    bj = 0x7fffffff;
#pragma unroll
                    for (int m = 0; m < MC; ++m) {
                        const int j = hl + HLN * m;
                        if (j < K) {
                            const bool seen = ((K1 || j < 64 ? t0 : t1) >> (j & 63)) & 1ULL;
                            const uint64_t key = seen ? ~0ULL : order_key(qv[m]);
                            if (key < bk) {  // lower m first: ties keep the lower index
                                bk = key;
                                bj = j;
                            }
                        }
                    }
                    auto take = [&](uint64_t ok, int oj) {
                        if (ok < bk || (ok == bk && oj < bj)) {
                            bk = ok;
                            bj = oj;
                        }
                    };
                    take(post_dpp64<0xB1>(bk), (int)post_dpp32<0xB1>((uint32_t)bj));
                    take(post_dpp64<0x4E>(bk), (int)post_dpp32<0x4E>((uint32_t)bj));
                    take(post_dpp64<0x141>(bk), (int)post_dpp32<0x141>((uint32_t)bj));
                    take(post_dpp64<0x140>(bk), (int)post_dpp32<0x140>((uint32_t)bj));
                    if constexpr (HLN == 32) take(pscl::shfl_u64(bk, lane ^ 16), __shfl(bj, lane ^ 16));
                };
                // exact sums: index order, each product and sum rounded (the oracle's restatement
                // of numpy's abs_l0 @ beta)
                auto sums_exact = [&]() {
#pragma unroll
                    for (int m = 0; m < MC; ++m) qv[m] = 0.0;
                    const double* bc = beta + hl;
#pragma unroll kSumUnroll
                    for (int k = 0; k < K; ++k) {
                        const double ak = nxt[k];
#pragma unroll
                        for (int m = 0; m < MC; ++m)
                            if (hl + HLN * m < K) qv[m] = qv[m] + ak * bc[k * K + HLN * m];
                    }
                };
                if (Q.beta && !(PSCL_POST_ABLATE & 4)) {
#if PSCL_POST_FMA
                    // screening sums with fused multiply-adds (half the VALU), then a certificate:
                    // |q_fma - q_exact| <= (gamma_64 + gamma_65) S, S = sum_k |L0_k| |beta_kj| <=
                    // ||L0||_1 max|beta|, so a best candidate whose screening sum is below every
                    // other untried candidate's by twice that bound is the exact (q, index) argmin;
                    // else the exact sums are recomputed (both halves: the certified one gets the
                    // same index back)
#pragma unroll
                    for (int m = 0; m < MC; ++m) qv[m] = 0.0;
                    constexpr bool PK = KC == 64;  // packed fp32 sums (narrow form, K = 64; e2 below)
                    if (MF && beta_lds == 2) {
                        // D[i][j] = sum_k beta[k][16 t + i] |L0_k| of entry slot j (j < 2), tile t = 0..3,
                        // on v_mfma_f32_16x16x4_f32: lane l gives A[l & 15][l >> 4] (a beta row) and
                        // B[l >> 4][l & 15] (the |L0| of slot l & 15, 0 for l & 15 >= 2); each output is
                        // the k-ordered fp32 fma chain of the packed path below, bit for bit
                        typedef float f4m __attribute__((ext_vector_type(4)));
                        const int jl = lane & 15, kl = lane >> 4;
                        // entry slot jl's fp32 |L0| (the same buffer parity as this lane's nxt)
                        const float* lj = reinterpret_cast<const float*>(S.lvl[wave][jl < 2 ? jl : 0][nxt == buf0 ? 0 : 1] + 64);
                        f4m acc[4];
#pragma unroll
                        for (int t = 0; t < 4; ++t) acc[t] = (f4m){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 2
                        for (int s4 = 0; s4 < 16; ++s4) {
                            const int k = 4 * s4 + kl;
                            const float bv = jl < 2 ? lj[k] : 0.0f;
#pragma unroll
                            for (int t = 0; t < 4; ++t)
                                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(sbeta32[k * 64 + ((16 * t + jl) ^ (16 * kl))], bv, acc[t], 0, 0, 0);
                        }
                        // D row 4 kl + r, column jl: candidate 16 t + 4 kl + r of slot jl, to LDS (doubles
                        // 96..127 of the slot's nxt: free until the tails), then each lane its own two
                        pscl::wave_lds_fence();  // (every lane's reads of the |L0| copies are done)
                        float* qj = reinterpret_cast<float*>(S.lvl[wave][jl < 2 ? jl : 0][nxt == buf0 ? 0 : 1] + 96);
                        if (jl < 2) {
#pragma unroll
                            for (int t = 0; t < 4; ++t)
#pragma unroll
                                for (int r = 0; r < 4; ++r) qj[16 * t + 4 * kl + r] = acc[t][r];
                        }
                        pscl::wave_lds_fence();
                        const float* qm = reinterpret_cast<const float*>(nxt + 96);
#pragma unroll
                        for (int m = 0; m < MC; ++m) qv[m] = (double)qm[hl + HLN * m];  // (exact widening)
                    } else if (PK && beta_lds == 2) {
                        // the lane's candidates in pairs, one v_pk_fma_f32 per pair and k: |L0| read 4 at
                        // a time (fp32 copy), beta from the lane layout; summed in fp32 and certified
                        // against the fp32 bound below (the exact fp64 sums when uncertified)
                        typedef float f2 __attribute__((ext_vector_type(2)));
                        typedef float f4 __attribute__((ext_vector_type(4)));
                        constexpr int NP = MC / 2;  // candidate pairs per lane
                        const f2* bp = reinterpret_cast<const f2*>(sbeta32) + hl * NP;
                        const f4* lp = reinterpret_cast<const f4*>(l32);
                        f2 acc[NP];
#pragma unroll
                        for (int i = 0; i < NP; ++i) acc[i] = (f2){0.0f, 0.0f};
#pragma unroll kPkUnroll
                        for (int k4 = 0; k4 < 16; ++k4) {
                            const f4 a = lp[k4];
#pragma unroll
                            for (int i = 0; i < NP; ++i) {
                                acc[i] = __builtin_elementwise_fma((f2){a.x, a.x}, bp[(4 * k4 + 0) * HLN * NP + i], acc[i]);
                                acc[i] = __builtin_elementwise_fma((f2){a.y, a.y}, bp[(4 * k4 + 1) * HLN * NP + i], acc[i]);
                                acc[i] = __builtin_elementwise_fma((f2){a.z, a.z}, bp[(4 * k4 + 2) * HLN * NP + i], acc[i]);
                                acc[i] = __builtin_elementwise_fma((f2){a.w, a.w}, bp[(4 * k4 + 3) * HLN * NP + i], acc[i]);
                            }
                        }
#pragma unroll
                        for (int i = 0; i < NP; ++i) {  // (exact widening; candidate m = 2 i, 2 i + 1)
                            qv[2 * i] = (double)acc[i].x;
                            qv[2 * i + 1] = (double)acc[i].y;
                        }
                    } else if (beta_lds == 2) {  // (narrow form: beta staged in LDS as fp32, see e2 below)
                        const float* bc = sbeta32 + hl;
#pragma unroll kSumUnroll
                        for (int k = 0; k < K; ++k) {
                            const double ak = nxt[k];
#pragma unroll
                            for (int m = 0; m < MC; ++m)
                                if (hl + HLN * m < K) qv[m] = __builtin_fma(ak, (double)bc[k * K + HLN * m], qv[m]);
                        }
                    } else {
                        const double* bc = beta + hl;
#pragma unroll kSumUnroll
                        for (int k = 0; k < K; ++k) {
                            const double ak = nxt[k];
#pragma unroll
                            for (int m = 0; m < MC; ++m)
                                if (hl + HLN * m < K) qv[m] = __builtin_fma(ak, bc[k * K + HLN * m], qv[m]);
                        }
                    }
                    argmin();
                    double as = 0.0;
#pragma unroll
                    for (int m = 0; m < MC; ++m) as = as + (hl + HLN * m < K ? nxt[hl + HLN * m] : 0.0);
                    as = as + pscl_asf64(post_dpp64<0xB1>(pscl_asu64(as)));
                    as = as + pscl_asf64(post_dpp64<0x4E>(pscl_asu64(as)));
                    as = as + pscl_asf64(post_dpp64<0x141>(pscl_asu64(as)));
                    as = as + pscl_asf64(post_dpp64<0x140>(pscl_asu64(as)));
                    if constexpr (HLN == 32) as = as + pscl_asf64(pscl::shfl_u64(pscl_asu64(as), lane ^ 16));
                    // 2 E = 2 (gamma_K + gamma_K+1) S <= (4 K + 2 + slack) u S, u = 2^-53 (K = 64:
                    // 264 u, 2.3 % slack; the bound grows with K, so the (128,88) and runtime-K
                    // instances get their own); fp32 beta adds |beta32 - beta| <= 2^-24 |beta| + 2^-150
                    // per term, i.e. 2^-24 S + 2^-150 ||L0||_1 (2 % slack on the doubled bound)
                    const double gk = (4.0 * (double)K + 8.0) * 0x1p-53;
                    // packed fp32 sums: |L0| and beta each rounded to fp32 (u = 2^-24 relative per
                    // factor, plus 2^-150 absolute where the value lands in fp32's subnormal range),
                    // K fp32 fma roundings (gamma_K, plus 2^-149 each in the subnormal range), the
                    // exact sums' own gamma_K (fp64):
                    //   |q32 - q_exact| <= ((K + 2.01) 2^-24 + gk / 2) S + K 2^-149
                    //                      + ||L0||_1 2^-150 + K max|beta| 2^-150
                    // (S <= ||L0||_1 max|beta|; the last two terms: a subnormal beta32 or |L0|32 times
                    // the other factor, summed over k); doubled, 2 % slack.  Trusted only when every
                    // |L0_k| and product is far inside fp32 range (||L0||_1 < 2^100 and ||L0||_1
                    // max|beta| < 2^100): a larger, infinite or NaN ||L0||_1 (an fp32 copy of inf, and
                    // inf * 0 = NaN sums) leaves the certificate false and the exact sums decide
                    const double e2 = (PK && beta_lds == 2)
                                          ? ((as < 0x1p100 && as * Q.beta_absmax < 0x1p100)
                                                 ? 2.04 * (as * Q.beta_absmax * (((double)K + 2.01) * 0x1p-24 + 0.5 * gk)
                                                           + (double)K * 0x1p-149 + as * 0x1p-150
                                                           + (double)K * Q.beta_absmax * 0x1p-150)
                                                 : __builtin_inf())
                                      : beta_lds == 2 ? as * Q.beta_absmax * (gk + 2.04 * 0x1p-24) + as * 0x1p-140
                                                      : as * Q.beta_absmax * gk;
                    double qmine = qv[0];
#pragma unroll
                    for (int m = 1; m < MC; ++m) qmine = (bj / HLN) == m ? qv[m] : qmine;
                    const double qb = pscl_asf64(pscl::shfl_u64(pscl_asu64(qmine), hb + (bj % HLN)));
                    const double thr = qb + e2 * (1.0 + 0x1p-40);
                    bool near = false;
#pragma unroll
                    for (int m = 0; m < MC; ++m) {
                        const int j = hl + HLN * m;
                        const bool seen = ((K1 || j < 64 ? t0 : t1) >> (j & 63)) & 1ULL;
                        near = near || (j < K && j != bj && !seen && !(qv[m] > thr));
                    }
                    if (__ballot(near && more) && !(PSCL_POST_ABLATE & 64)) {
                        sums_exact();
                        argmin();
                    }
#else
                    sums_exact();
                    argmin();
#endif
                } else {
#pragma unroll
                    for (int m = 0; m < MC; ++m) qv[m] = hl + HLN * m < K ? nxt[hl + HLN * m] : 0.0;
                    argmin();
                }
                const int idx = bj;  // (half-uniform) an untried index exists: rounds <= min(retries, K)
                // the 16-phase block of its position (info_set[idx] >> 4): blocks whose cumulative
                // information-bit count is at most idx (no memory read)
                int seg = 0;
#pragma unroll
                for (int b = 0; b < PSCL_DL_NSEG - 1; ++b) seg += (idx < K && icum[b] <= idx) ? 1 : 0;
                if (PSCL_POST_ABLATE & 2) seg = 0;
                pscl::wave_lds_fence();  // (the select's reads of nxt before the tails overwrite it)
                // ---- exact metric increments of the forced prefix's leaves (scl.py:102-105, as
                // the decode kernel forms them: good child metric + L, bad child metric +
                // (|llr| + L), llr == 0: metric + LOGE2), then summed in phase order
                // (Q.warm_apx: the screening tail, PSCL_TUNE_DL_WARM_APX -- a screened decode's own)
                auto tails = [&](auto tailf) {
#pragma unroll
                    for (int m = 0; m < EL; ++m) {
                        const int p = hl + HLN * m;
                        if (p < 16 * seg) {
                            const double lam = RR ? lv[m] : cur[p];  // (the leaves: lv[], or in cur)
                            const uint32_t bit = (uint32_t)(((p < 64 ? u0 : u1) >> (p & 63)) & 1ULL);
                            const double Lt = tailf(lam);
                            const bool good = bit == (lam < 0.0 ? 1u : 0u);
                            nxt[p] = lam == 0.0 ? PSCL_LOGE2 : (good ? Lt : fabs(lam) + Lt);
                        }
                    }
                };
                if (Q.warm_apx)
                    tails([](double v) { return pscl_softplus_tail_abs(v); });
                else
                    tails([&](double v) { return pscl_softplus_tail_bf(v, S.exp_table); });
                pscl::wave_lds_fence();
                if (Q.warm_apx) {
                    // screening warm metrics (any summation order: the screened decode's relative
                    // slack covers it): the 16-phase blocks summed in parallel, lane b block b,
                    // into cur (its leaves are read)
                    if (hl < seg) {
                        double bsum = 0.0;
#pragma unroll
                        for (int qq = 0; qq < 16; ++qq) bsum = bsum + nxt[16 * hl + qq];
                        cur[hl] = bsum;
                    }
                    pscl::wave_lds_fence();
                }
                if (more && hl == 0) {
                    double mt = 0.0;
                    double* wm = Q.warm_metric + (int64_t)e * PSCL_DL_NSEG;
                    if (Q.warm_apx) {
                        for (int k = 0; k <= seg; ++k) {
                            wm[k] = mt;
                            if (k < seg) mt = mt + cur[k];
                        }
                    } else {  // exact: in phase order, as the exact decode accumulates them
                        for (int k = 0; k <= seg; ++k) {
                            wm[k] = mt;
                            if (k < seg && !(PSCL_POST_ABLATE & 8))
                                for (int qq = 0; qq < 16; ++qq) mt = mt + nxt[16 * k + qq];
                        }
                    }
                    Q.warm_u[2 * e] = u0;
                    Q.warm_u[2 * e + 1] = u1;
                    // tried set, flip record
                    Q.tried[2 * e] = idx < 64 ? (t0 | (1ULL << idx)) : t0;
                    Q.tried[2 * e + 1] = idx >= 64 ? (t1 | (1ULL << (idx - 64))) : t1;
                    Q.ntried[e] = nt + 1;
                    if (Q.tried_out) Q.tried_out[f * Q.tried_stride + nt] = idx;
                    // _force_vector (flip.py:30-34): bits [0, idx) = reference, bit idx flipped, rest free
                    uint64_t* fr = Q.force + (int64_t)e * 2 * W;
                    for (int w = 0; w < W; ++w) {
                        const int lo = 64 * w;
                        const int nb = idx - lo + 1;  // bits of this word in [0, idx]
                        const uint64_t mask = nb <= 0 ? 0ULL : (nb >= 64 ? ~0ULL : ((1ULL << nb) - 1ULL));
                        uint64_t val = (w ? b1 : b0) & mask;
                        if (idx >= lo && idx < lo + 64) val ^= 1ULL << (idx - lo);
                        fr[w] = mask;
                        fr[W + w] = val;
                    }
                    // staged append to bucket seg of the next round (LDS atomics)
                    const int sl = atomicAdd(&S.nst, 1);
                    S.st_e[sl] = e;
                    S.st_seg[sl] = (uint8_t)seg;
                    S.st_pos[sl] = (uint16_t)atomicAdd(&S.lcnt[seg], 1);
                }
                pscl::wave_lds_fence();  // the LDS buffers are rewritten by the next pair
            }
        }
        // flush: one global atomic per non-empty bucket, then the staged entries scattered
        // (tid opaque: the flush's thread-indexed addresses are formed here, not hoisted out of
        // the entry loop into registers held across it)
        int tid = (int)threadIdx.x;
        asm volatile("" : "+v"(tid));
        __syncthreads();
        if (tid < PSCL_DL_NSEG) {
            const int cc = S.lcnt[tid];
            int g = 0;
            if (cc) {
                if (PSCL_POST_ABLATE & 1) g = 0;
                else g = atomicAdd(Q.out_count + tid * PSCL_DL_CSTRIDE, cc);
            }
            S.gbase[tid] = g;
        }
        __syncthreads();
        const int nst = S.nst;
        for (int x = tid; x < nst; x += (int)blockDim.x) {
            const int sg = S.st_seg[x];
            Q.out_list[(int64_t)sg * Q.cap + S.gbase[sg] + S.st_pos[x]] = S.st_e[x];
        }
        __syncthreads();
        if (tid < PSCL_DL_NSEG) S.lcnt[tid] = 0;
        if (tid == 0) S.nst = 0;
        __syncthreads();
    }
    if (Q.counters && decodes)
        atomicAdd(reinterpret_cast<unsigned long long*>(Q.counters) + PSCL_CNT_RETRIES, decodes);
}

// Post pass of the long codes (N > PSCL_FAST_N): one wavefront per entry, no replay -- the
// retry decodes run the HIST kernel, so the attempt's best-path decision LLRs (L0, scl.py:158,
// 166) arrive with it.  Per entry: final-attempt bookkeeping and the CRC stop rule
// (flip.py:123-136); for the survivors the next flip (q = |L0| @ beta summed in index order,
// argmin over untried (q, index), flip.py:104-111), its force words (flip.py:30-34), and the
// entry's state moved to a dense slot of the next pass (one atomic per wavefront).  The long
// kernel decodes every phase, so there is no warm start.
__global__ void __launch_bounds__(256) dl_post_long_kernel(const pscl_post_long_params Q) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int K = Q.K, W = Q.W;
    const int64_t n_in = *Q.in_count < Q.cap ? (int64_t)*Q.in_count : Q.cap;
    const int64_t wstride = (int64_t)gridDim.x * (blockDim.x >> 6);
    unsigned long long decodes = 0;
    for (int64_t e = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave; e < n_in; e += wstride) {  // wave-uniform
        const int64_t f = Q.act_in[e];
        const int nt = Q.init ? 0 : Q.nt_in[e];
        const uint8_t fl = Q.of[e];
        const uint64_t* bw = Q.ob + e * W;
        bool more;
        if (Q.init) {  // baseline failing by construction (dl_compact); its results stay
            more = Q.rounds > 0;
        } else {       // the attempt just decoded is the frame's latest
            for (int w = lane; w < W; w += 64) Q.best[f * W + w] = bw[w];
            if (lane == 0) {
                Q.flags[f] = fl;
                if (Q.attempts) Q.attempts[f] = nt + 1;
            }
            ++decodes;
            more = !(fl & PSCL_FLAG_CRC_PASS) && nt < Q.rounds;
        }
        if (!more) continue;
        // next flip: candidates j = lane + 64 m, q_j summed over k in index order
        const double* a = Q.l0 + e * K;
        uint64_t bk = ~0ULL;
        int bj = 0x7fffffff;
        for (int j0 = 0; j0 < K; j0 += 64) {
            const int j = j0 + lane;
            double q = 0.0;
            if (j < K) {
                if (Q.beta) {
                    for (int k = 0; k < K; ++k) q = q + fabs(a[k]) * Q.beta[(int64_t)k * K + j];
                } else {
                    q = fabs(a[j]);
                }
                const bool seen = !Q.init && ((Q.tried_in[e * W + (j >> 6)] >> (j & 63)) & 1ULL);
                const uint64_t key = seen ? ~0ULL : order_key(q);
                if (key < bk) {  // lower j first: ties keep the lower index
                    bk = key;
                    bj = j;
                }
            }
        }
#pragma unroll
        for (int sft = 1; sft < 64; sft <<= 1) {  // wave argmin of (key, index)
            const uint64_t ok = pscl::shfl_u64(bk, lane ^ sft);
            const int oj = __shfl(bj, lane ^ sft);
            if (ok < bk || (ok == bk && oj < bj)) {
                bk = ok;
                bj = oj;
            }
        }
        const int idx = bj;  // an untried index exists: rounds <= min(retries, K)
        int slot = 0;
        if (lane == 0) slot = atomicAdd(Q.out_count, 1);
        const int64_t e2 = __shfl(slot, 0);
        if (lane == 0) {
            Q.act_out[e2] = f;
            Q.nt_out[e2] = nt + 1;
            if (Q.tried_out) Q.tried_out[f * Q.tried_stride + nt] = idx;
        }
        for (int w = lane; w < W; w += 64) {
            const uint64_t t = Q.init ? 0ULL : Q.tried_in[e * W + w];
            Q.tried_w_out[e2 * W + w] = (idx >> 6) == w ? (t | (1ULL << (idx & 63))) : t;
            // _force_vector (flip.py:30-34): bits [0, idx) = reference, bit idx flipped, rest free
            const int lo = 64 * w, nb = idx - lo + 1;
            const uint64_t mask = nb <= 0 ? 0ULL : (nb >= 64 ? ~0ULL : ((1ULL << nb) - 1ULL));
            uint64_t val = bw[w] & mask;
            if (idx >= lo && idx < lo + 64) val ^= 1ULL << (idx - lo);
            Q.force[e2 * 2 * W + w] = mask;
            Q.force[e2 * 2 * W + W + w] = val;
        }
    }
    if (Q.counters && lane == 0 && decodes)
        atomicAdd(reinterpret_cast<unsigned long long*>(Q.counters) + PSCL_CNT_RETRIES, decodes);
}

// FER/BER statistics of the final results against the transmitted words: per-thread sums over a
// grid stride, wavefront sums, then one atomic per counter per 256-thread block.  (Blocks of 1024
// threads -- 16 wavefronts that must start on one CU together -- waited up to ~350 us for a CU to
// drain beside the next call's baseline decode in the pipelined sweep, r06m.)
__global__ void __launch_bounds__(256) dl_count_kernel(const uint64_t* __restrict__ best, const uint8_t* __restrict__ flags,
                                                       const uint64_t* __restrict__ ref, int64_t B, int W, int k_payload,
                                                       int64_t* counters) {
    __shared__ int part[4][4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned long long* C = reinterpret_cast<unsigned long long*>(counters);
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(C + PSCL_CNT_FRAMES, (unsigned long long)B);
    int v[4] = {0, 0, 0, 0};  // frame errors, bit errors, payload frame errors, payload bit errors
    for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < B; f += (int64_t)gridDim.x * blockDim.x) {
        v[0] += (flags[f] & PSCL_FLAG_CRC_PASS) ? 0 : 1;
        int be = 0, pb = 0;
        for (int w = 0; w < W; ++w) {  // payload = the first k_payload information bits
            const uint64_t d = best[f * W + w] ^ ref[f * W + w];
            const int kp = k_payload - 64 * w;
            const uint64_t pm = kp >= 64 ? ~0ULL : (kp > 0 ? ((1ULL << kp) - 1) : 0ULL);
            be += __popcll(d);
            pb += __popcll(d & pm);
        }
        v[1] += be;
        v[2] += pb ? 1 : 0;
        v[3] += pb;
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

hipError_t pscl_launch_dl_post_long(const pscl_post_long_params& Q, hipStream_t s) {
    if (Q.cap <= 0) return hipSuccess;
    int64_t grid = (Q.cap + 3) / 4;  // one wavefront per entry, the live count read on the device
    if (grid > 2048) grid = 2048;
    hipLaunchKernelGGL(dl_post_long_kernel, dim3((unsigned)grid), dim3(256), 0, s, Q);
    return hipGetLastError();
}

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

hipError_t pscl_launch_replay(const pscl_replay_params& R, int64_t cap, hipStream_t s) {
    if (cap <= 0) return hipSuccess;
    const int64_t grid = (cap + 3) / 4;
    hipLaunchKernelGGL(replay_kernel, dim3((unsigned)grid), dim3(256), 0, s, R, cap);
    return hipGetLastError();
}

// entries per wavefront of the launch (the 4-entry form is instantiated for the (128,64) code: its
// K = 64 sums fit 3 wavefronts per SIMD without spills; others run 2 entries per wavefront)
int pscl_post_epw(const pscl_post_params& Q) {
    if (!Q.narrow) return kPostEpwWide;
    if (!(Q.N == 128 && Q.K == 64)) return 2;
    return Q.epw == 2 || Q.epw == 4 ? Q.epw : kPostEpwNarrow;
}

hipError_t pscl_launch_dl_post(const pscl_post_params& Q, int64_t entries, hipStream_t s) {
    if (entries <= 0) return hipSuccess;
    // workgroups of PW wavefronts (EPW PW entries in flight), sized for `pairs` iterations per wavefront
    const int PW = Q.narrow ? kPostWavesNarrow : kPostWavesWide;
    const int EPW = pscl_post_epw(Q);
    const int64_t pairs = Q.pairs >= 1 && Q.pairs <= 32 ? Q.pairs : PSCL_POST_PAIRS;
    int64_t grid = (entries + PW * EPW * pairs - 1) / (PW * EPW * pairs);
    const int64_t gcap = Q.grid_cap >= 16 && Q.grid_cap <= 4096 ? Q.grid_cap : PSCL_POST_GRID;  // (tuning knob)
    if (grid > gcap) grid = gcap;
    // beta in LDS: fp64 in the wide form (LDS <= 64 KB), fp32 in the narrow one (16 KB at K = 64, beside
    // the next call's baseline; its rows read through L2 lost to that baseline's streaming: the flip
    // metric measured 48 of 109 us per pass, profiles/r04p2_post_trace.txt)
    const int beta_lds = !Q.beta ? 0
                         : (PSCL_POST_BETA_LDS && !Q.narrow && (size_t)Q.K * Q.K * 8 <= 32 * 1024) ? 1
                         : (PSCL_POST_BETA32 && Q.narrow && (size_t)Q.K * Q.K * 4 <= 16 * 1024) ? 2 : 0;
    const size_t lds = beta_lds == 1 ? (size_t)Q.K * Q.K * 8 : beta_lds == 2 ? (size_t)Q.K * Q.K * 4 : 0;
    const dim3 g((unsigned)grid), b(PW * 64);
    if (Q.narrow && EPW == 4) {
        hipLaunchKernelGGL((dl_post_kernel<128, 64, kPostWavesNarrow, 4>), g, b, lds, s, Q, beta_lds);
    } else if (Q.narrow) {
        if (Q.N == 128 && Q.K == 64)
            hipLaunchKernelGGL((dl_post_kernel<128, 64, kPostWavesNarrow, 2>), g, b, lds, s, Q, beta_lds);
        else if (Q.N == 128 && Q.K == 88)
            hipLaunchKernelGGL((dl_post_kernel<128, 88, kPostWavesNarrow, 2>), g, b, lds, s, Q, beta_lds);
        else
            hipLaunchKernelGGL((dl_post_kernel<0, 0, kPostWavesNarrow, 2>), g, b, lds, s, Q, beta_lds);
    } else if (Q.N == 128 && Q.K == 64) {
        hipLaunchKernelGGL((dl_post_kernel<128, 64, kPostWavesWide, kPostEpwWide>), g, b, lds, s, Q, beta_lds);
    } else if (Q.N == 128 && Q.K == 88) {
        hipLaunchKernelGGL((dl_post_kernel<128, 88, kPostWavesWide, kPostEpwWide>), g, b, lds, s, Q, beta_lds);
    } else {
        hipLaunchKernelGGL((dl_post_kernel<0, 0, kPostWavesWide, kPostEpwWide>), g, b, lds, s, Q, beta_lds);
    }
    return hipGetLastError();
}

hipError_t pscl_launch_dl_count(const uint64_t* best, const uint8_t* flags, const uint64_t* ref, int64_t B, int W,
                                int k_payload, int64_t* counters, hipStream_t s) {
    int64_t grid = (B + 1023) / 1024;  // (four frames per thread)
    if (grid > 1024) grid = 1024;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(dl_count_kernel, dim3((unsigned)grid), dim3(256), 0, s, best, flags, ref, B, W, k_payload,
                       counters);
    return hipGetLastError();
}
