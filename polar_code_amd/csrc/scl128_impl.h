#ifndef PSCL_SCL128_IMPL_H
#define PSCL_SCL128_IMPL_H
// scl128_impl.h -- the specialised list decoder kernel (included by scl128.hip and
// scl128_spec*.hip, which instantiate and launch it).  Specialised list decoder for N = 128 and list sizes L <= 8 (every BASELINE
// configuration).  Same contract and bit-exact results as the generic kernel in
// scl_kernels.hip (decode_scl, dl_scl_polar/polar/scl.py:108-209); the N = 128 shape is
// compiled in so the tree walk is straight-line code.
//
// Wavefront layout: F = 64/G frames per wavefront, G = 2*LMAX lanes per frame.  Lane g < L
// of a frame group holds list path g (metric, list position `rank`, decided bits u, and the
// LDS slot of each stored depth); lane g + LMAX is that path's bit-1 child while the list is
// extended, and otherwise evaluates the sibling leaf's metric tail (below).
//
// LLR tree, per frame in LDS: (with rate matching) the 128 channel LLRs and, per path slot, depths 3..6
// (16 + 8 + 4 + 2 values).  Depths 1 and 2 are never stored: every 16th phase the lanes
// recompute the 16 depth-3 values of each path directly from 8 channel LLRs each (f/g through
// depths 1-3), which halves the LDS footprint per frame and with it raises occupancy.
//
// List update per phase:
//   frozen  (all paths take bit 0, scl.py:149-153): metrics advance and the stable order is
//           re-ranked in place (rank on (metric, rank)); no path state moves.
//   info    (free, forced or SC-hard): 2L children ranked on (metric, 2*rank + bit) with a
//           rotation count (python's stable sort, scl.py:173), survivors gathered into lanes
//           0..L-1 in list order (scl.py:174).
// Metric tail: at a frozen even leaf the right sibling's LLR for the known left bit is
// already fixed, so lanes g >= LMAX evaluate its log1p(exp(-|llr|)) in the same pass; the
// next phase reuses it (48 of 128 evaluations per frame for the (128,64) code).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "glibc_softplus.h"
#include "scl_device.h"
#include "scl_kernels.h"

namespace {

using namespace pscl;

// a wavefront's error counts at the end of a counting launch: stored at its slot of P.cpart, or
// added to P.counters with one atomic per counter (flush_counts)
// (P.cpart is all zero between launches -- zeroed when allocated and by the reduce that reads it --
// so a wavefront without errors, most of them at the SNRs of interest, stores nothing)
__device__ __forceinline__ void flush_counts_p(const pscl_decode_params& P, int64_t wslot, int fe, int be, int pe, int pb) {
    if (P.cpart) {
        if (!__builtin_amdgcn_ballot_w64((fe | be | pe | pb) != 0)) return;
        fe = wave_sum(fe);
        be = wave_sum(be);
        pe = wave_sum(pe);
        pb = wave_sum(pb);
        if ((threadIdx.x & 63) == 0) reinterpret_cast<int4*>(P.cpart)[wslot] = make_int4(fe, be, pe, pb);
    } else {
        flush_counts(P.counters, fe, be, pe, pb);
    }
}

constexpr int kN = 128;
constexpr int kn = 7;

// 16-lane frames keep their 8 channel LLRs in registers across the depth-1..3 recomputes
#ifndef PSCL_CREG
#define PSCL_CREG 1
#endif

// CH: the frame's channel LLRs are staged in LDS (needed when the decode input is rate
// matched: the de-rate-matched values exist nowhere else); otherwise the depth-1..3
// recomputes read them straight from the (L2/MALL-resident) input row, which halves the
// LDS per frame and lets the wave count reach the register limit.
template <int LMAX, bool CH>
struct Layout128 {
    static constexpr int G = 2 * LMAX;
    static constexpr int F = 64 / G;
    static constexpr int LOG_G = __builtin_ctz(G);
    static constexpr int LOG_LM = __builtin_ctz(LMAX);
    // 16-lane frames (L = 8) hold their channel LLRs in registers (creg) from the frame's start:
    // a staged (CH) channel row is dead once loaded, so depth 3 is laid over it (the first
    // depth-3 write, at phase 0, follows the register loads) -- 2 KB per frame instead of 3 KB,
    // 4 waves/SIMD instead of 3 for the rate-matched NR decode
    static constexpr bool CREG = G == 16 && PSCL_CREG;
    // depth-d nodes (W = 2^(7-d) values per slot) pair-major, [W/2][slot][2]: element e of
    // slot s at ((e mod W/2) * LMAX + s) * 2 + e div W/2, so the two inputs a = e, b = e + W/2
    // of every f/g of the next depth (and of the leaf) are one 16-byte ds_read_b128 (4 LDS
    // cycles per wave, against 8 for the ds_read2_b64 of two separate doubles), and the
    // 16 lanes of a frame, each on its own path, read 256 contiguous bytes
    static constexpr int OFF3 = CH && !CREG ? kN : 0;  // [8][LMAX][2]
    static constexpr int OFF4 = OFF3 + 16 * LMAX;   // [4][LMAX][2]
    static constexpr int OFF5 = OFF4 + 8 * LMAX;    // [2][LMAX][2]
    static constexpr int OFF6 = OFF5 + 4 * LMAX;    // [1][LMAX][2]
    // the paths' left-sibling partial sums {X1 lo, X1 hi, X2, X2 >> 16 | X3 << 16} at a depth-1..3 recompute,
    // 16 B per path: every lane reads them for all paths with ds_read_b128
    static constexpr int OFFX = OFF6 + 2 * LMAX;
    // doubles per frame, padded to 256 B: the frames of a wave then start on bank 0.  (With 8-lane
    // frames, L = 4, every frame then uses the same 32 banks: 55 % of that kernel's LDS cycles are
    // bank conflicts.  PSCL_L128_PAD = 1 offsets frames narrower than 16 lanes by one access
    // footprint, 2 G doubles: conflicts 55 -> 37 %, but config 4 measured 3.64-3.68 ms per step
    // against 3.46-3.48 -- the larger LDS per wavefront costs more beside the retry chains than
    // the conflicts do -- profiles/r04j_l128_pad_ab.txt)
#ifndef PSCL_L128_PAD
#define PSCL_L128_PAD 0
#endif
    static constexpr int FSTRIDE = ((OFFX + 2 * LMAX + 31) & ~31) + (PSCL_L128_PAD && G < 16 ? 2 * G : 0);
    // position of element e of slot s in a node of width w
    static constexpr __device__ __forceinline__ int at(int w, int e, int s) {
        return ((e & (w / 2 - 1)) * LMAX + s) * 2 + e / (w / 2);
    }
};

__device__ __forceinline__ int slot_at(uint32_t tab, int d) { return (int)((tab >> (4 * (d - 3))) & 15u); }

// Arikan transform of the w-bit segment u[lo, lo+w), w <= 64, lo a multiple of w
__device__ __forceinline__ uint64_t seg_transform(uint64_t u0, uint64_t u1, int lo, int w) {
    const uint64_t word = lo >= 64 ? u1 : u0;
    const uint64_t seg = (w == 64) ? word : (word >> (lo & 63)) & ((1ULL << w) - 1);
    return polar_transform64(seg);
}

// depth-D step (D = 4, 5, 6) of the tree walk.  Lane (frame, g) works on path p = g mod LMAX
// of its own frame and the elements e = 2k + h (h = g / LMAX) of the node's W values, so the
// parent slot comes from the path's own slot table (tabp: upper lanes hold a copy) and no
// lane reads another's state.  Inputs e and e + W of the parent are one pair (Layout128).
//
// Addresses: with e = 2k + h, input pair e of slot s sits at double2 (2k LMAX) + (h LMAX + s)
// and (depths 4, 5) output element e of slot p at double 4k LMAX + 2 (h LMAX + p) (first half,
// 2k < W/2) or 2 (2k - W/2) LMAX + 1 + 2 (h LMAX + p): one per-lane base, lb = Af + 2 (h LMAX + p)
// doubles (= Af + 2g), serves every depth with compile-time offsets (depth 6 writes at 2p + h).
// Spelled out so the compiler keeps one base register instead of hoisting a dozen per-depth
// addresses out of the frame loop (register pressure sets the wave count).
template <int LMAX, bool CH, int D>
__device__ __forceinline__ void step_depth(double* Af, const double* lb, int g, uint32_t tabp, uint32_t xsp, bool first,
                                           bool is_g) {
    using Ly = Layout128<LMAX, CH>;
    constexpr int LW = kn - D, W = 1 << LW, HW = W / 2;
    constexpr int OFF_OUT = D == 4 ? Ly::OFF4 : (D == 5 ? Ly::OFF5 : Ly::OFF6);
    constexpr int OFF_IN = D == 4 ? Ly::OFF3 : (D == 5 ? Ly::OFF4 : Ly::OFF5);
    const int p = g & (LMAX - 1), h = g >> Ly::LOG_LM;
    // input base: the parent's slot (from the table at the first rewritten depth, else own)
    const double* in = first ? Af + 2 * (h * LMAX + slot_at(tabp, D - 1)) : lb;
    const uint32_t xh = xsp >> h;
    auto node = [&](int k) {  // element e = 2k + h
        const double2 ab = *reinterpret_cast<const double2*>(in + OFF_IN + 4 * k * LMAX);
        return is_g ? g_node(ab.x, ab.y, (xh >> (2 * k)) & 1u) : f_minsum(ab.x, ab.y);
    };
    if constexpr (D == 6) {
        Af[OFF_OUT + 2 * p + h] = node(0);
    } else {
        // the lane owns both members e, e + W/2 of each of its output pairs: one 16-byte store
        // per pair, the 16 lanes of a frame on 256 contiguous bytes (single-double stores at a
        // 16-byte stride put lanes g and g + 8 on the same banks)
#pragma unroll
        for (int k = 0; k < HW / 2; ++k)
            *reinterpret_cast<double2*>(const_cast<double*>(lb) + OFF_OUT + 4 * k * LMAX) = make_double2(node(k), node(k + HW / 2));
    }
    wave_lds_fence();
}

// Information sets compiled into dedicated kernels: construct_info_set(128, 64) and
// construct_info_set(128, 88) (polar.py:85-103, design SNR 2.5 dB) -- BASELINE configs 1-4 and
// the NR config 5.  Bit phi set <=> phase phi carries information.  Any other set runs the
// CODE = 0 kernels with the mask from the launch.
__device__ constexpr uint64_t kSpecInfo[3][2] = {
    {0, 0},
    {0xeee8e888e8a8a880ULL, 0xfeeaeee8eee8e880ULL},
    {0xfeeaeee8fee8e888ULL, 0xfffefeeafeeaeee8ULL},
};
constexpr int kSpecK[3] = {0, 64, 88};

template <typename Fn, int... I>
__device__ __forceinline__ void static_for_impl(Fn& fn, std::integer_sequence<int, I...>) {
    (fn(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
    static_for_impl(fn, std::make_integer_sequence<int, N>{});
}

// info phases rank the 2L children on the metric alone and fall back to the full tie key
// only when equal metrics leave a list position unclaimed
#ifndef PSCL_RANK_M
#define PSCL_RANK_M 1
#endif

// Timing-only ablations of the screening kernel (tools/build_variant.py --spec 1_8
// -DPSCL_APX_ABLATE=m); 0 in the product.  1: tail -> |lam| * 2^-20; 2: no depth-1..3
// recompute; 4: no depth-4..6 steps; 8: full-list info phases always take the fast path;
// 16: no final-order certification; 32: full-list info phases always rank
#ifndef PSCL_APX_ABLATE
#define PSCL_APX_ABLATE 0
#endif

#ifndef PSCL_LEAF_BLEND
#define PSCL_LEAF_BLEND 0
#endif

// L >= 4 screening: the metric tail without the |v| clamp; frames whose channel magnitudes could
// push a tree LLR to 2^30 are deferred (the check at the frame's start, below)
#ifndef PSCL_TAIL_NC
#define PSCL_TAIL_NC 1
#endif

// diagnostic builds only: the history instances with the aggregated counters (docs/HISTORY.md §5.6)
#ifndef PSCL_HIST_AGG
#define PSCL_HIST_AGG 0
#endif
#ifndef PSCL_WAVES_PER_EU
#define PSCL_WAVES_PER_EU 4
#endif
// the exact plain and forced-bit instances (the re-decode of deferred frames, the DL-SCL retry
// decodes: few frames per launch, latency-bound): 3 waves/SIMD, i.e. up to 168 VGPRs -- at 4
// (128 VGPRs) they spilled 4-16 VGPRs and 20-60 B per lane to scratch, and a kernel with scratch
// makes the runtime (re)allocate a queue's scratch at its first launch there (a ~130 us dispatch
// stall measured on a retry stream, rocprofv3 scratch-memory trace)
#ifndef PSCL_EXACT_WAVES_PER_EU
#define PSCL_EXACT_WAVES_PER_EU 3
#endif

// FS: the launch may carry forced bits or SC hard decisions (P.force / P.sc_hard).  Without
// them (every plain SCL decode) the per-frame force words and their tests compile away.
// APX: screening decode (plain decodes of the compiled-in codes): metric tails from the
// bounded-error pscl_softplus_tail_scr; every ordering decision is made on the metrics' high
// words and must clear a margin of PSCL_SCR_H units (glibc_softplus.h: proven to exceed twice
// the metric error), else the frame is appended to P.amb_list for an exact re-decode.
template <int LMAX, bool HIST, bool CH, bool FS, int CODE, bool APX = false>
__global__ void __launch_bounds__(PSCL_MAX_WAVES_PER_WG * 64)
__attribute__((amdgpu_waves_per_eu((APX || HIST) ? PSCL_WAVES_PER_EU : PSCL_EXACT_WAVES_PER_EU)))
scl128_kernel(const pscl_decode_params P) {
    using Ly = Layout128<LMAX, CH>;
    const uint64_t* const force = FS ? P.force : nullptr;
    const bool sc_hard = FS && P.sc_hard;
    constexpr int G = Ly::G, F = Ly::F, LOG_G = Ly::LOG_G;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t* T = reinterpret_cast<uint64_t*>(smem);
    // the exp table of the exact metric tail (the screening tail needs none: pscl_decode_layout
    // leaves it out of the screening launch's LDS)
    constexpr int TW = APX ? 0 : PSCL_EXP_TABLE_WORDS;
    for (int i = threadIdx.x; i < TW; i += blockDim.x) T[i] = P.exp_table[i];
#if PSCL_EPI_LDS
    for (int i = threadIdx.x; i < P.epi_words; i += blockDim.x) T[TW + i] = P.epi_table[i];
    const uint8_t* GT = reinterpret_cast<const uint8_t*>(T + TW);  // [16][256]
#else  // epilogue tables read from global memory (L1/L2-resident): less LDS per workgroup
    const uint8_t* GT = reinterpret_cast<const uint8_t*>(P.epi_table);
#endif
    __syncthreads();
    const uint32_t* ST = reinterpret_cast<const uint32_t*>(GT + 16 * 256);           // [K4][16]

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int fl = lane >> LOG_G;
    const int g = lane & (G - 1);
    const int gbase = lane & ~(G - 1);
    // with a compiled-in information set and no forced bits the list is full-size (launches
    // with L != LMAX take the CODE 0 kernels) and its length at every phase is known
    constexpr bool kFixedList = CODE != 0 && !FS;
    // K and the word count W are compile-time constants with a compiled-in code (the epilogue's
    // syndrome lookups then unroll with immediate LDS offsets)
    const int K = CODE ? kSpecK[CODE] : P.K, L = kFixedList ? LMAX : P.L;
    const int PW = CODE ? (kSpecK[CODE] + 63) / 64 : P.W;
    unsigned char* wbase = smem + P.wg_fixed_bytes + (size_t)wave * P.wave_bytes;
    double* A = reinterpret_cast<double*>(wbase);
    double* Af = A + fl * Ly::FSTRIDE;
    double* hist_llr = reinterpret_cast<double*>(wbase + P.a_bytes) + (size_t)fl * K * L;
    uint8_t* hist_par = wbase + P.a_bytes + (size_t)F * K * L * 8 + (size_t)fl * K * L;

    const int wpg = (int)(blockDim.x >> 6);
    const int64_t wstride = (int64_t)gridDim.x * wpg * F;
    const bool path_lane = g < LMAX;
    const int cpath = g & (LMAX - 1);
    const uint32_t cbit = g >= LMAX ? 1u : 0u;
    // information set: compiled in for the BASELINE codes (CODE 1, 2), else the launch's mask
    const uint64_t info0 = CODE ? kSpecInfo[CODE][0] : P.info_mask[0];
    const uint64_t info1 = CODE ? kSpecInfo[CODE][1] : P.info_mask[1];

    // live batch size: P.B, or a device-side count bounded by P.B, or (DL-SCL retry rounds)
    // the total of the bucket lists
    int bpre[PSCL_DL_NSEG + 1];
    const bool elist = FS && P.elist;
    int64_t Bn = P.d_count ? (*P.d_count < P.B ? (int64_t)*P.d_count : P.B) : P.B;
    if (elist) {
        const int64_t tot = pscl_bucket_prefix(P.bcount, P.bcap, bpre);
        Bn = tot < P.B ? tot : P.B;
    }
    int cfe = 0, cbe = 0, cpe = 0, cpb = 0;  // this lane's error counts (flushed at the end)
    for (int64_t f0 = ((int64_t)blockIdx.x * wpg + wave) * F; f0 < Bn; f0 += wstride) {
        const int64_t fi = f0 + fl;
        const bool fvalid = fi < Bn;
        const int64_t fsafe = fvalid ? fi : f0;
        // f indexes the force words and the outputs: the launch's frame index, or the entry id
        // of a bucket-list launch (then also the LLR row's index in fidx)
        int64_t f = fi;
        int seg0 = 0;  // warm start: first 16-phase segment decoded (wave-uniform)
        if (elist) {
            f = pscl_elist_entry(P, fsafe, bpre);
            seg0 = pscl_bucket_of(f0, bpre);
        }
        const int64_t frow = P.fidx ? P.fidx[elist ? f : fsafe] : fsafe;
        const double* chan = P.llr + frow * kN;  // !CH: channel LLRs read in place
        if (CH) {
            if (P.rm_E == 0) {
#pragma unroll
                for (int x = 0; x < kN / G; ++x) Af[g + x * G] = chan[g + x * G];
            } else {  // NR: de-rate-match + de-interleave while staging
                const double* src = P.llr + frow * P.rm_E;
                for (int x = 0; x < kN / G; ++x) Af[g + x * G] = nr_stage(src, P.rm_src[g + x * G], P.rm_E, kN);
            }
        }
        // 16-lane frames (L = 8): lane g's 8 channel LLRs (elements g + 16 m) are the same at
        // all 8 depth-1..3 recomputes: loaded once per frame into registers, so the recomputes
        // wait on no memory (16 VGPRs; the in-place reads cost 25 % of the screening pass)
        constexpr bool CREG = Ly::CREG;
        double creg[CREG ? 8 : 1];
        if constexpr (CREG) {
            if (CH) wave_lds_fence();
#pragma unroll
            for (int m = 0; m < 8; ++m) creg[m] = CH ? Af[g + 16 * m] : chan[g + 16 * m];
        }
        uint64_t fm0 = 0, fm1 = 0, fv0 = 0, fv1 = 0;
        if (FS && force && fvalid) {
            const uint64_t* fr = force + f * 2 * PW;
            fm0 = fr[0];
            fv0 = fr[PW];
            if (PW > 1) {
                fm1 = fr[1];
                fv1 = fr[PW + 1];
            }
        }
        wave_lds_fence();
        double metric = 0.0;
        uint32_t rank = 0;          // list position of this path
        uint64_t u0 = 0, u1 = 0;    // decided bits
        if constexpr (FS && CODE != 0) {
            // warm start at phase 16 seg0: the forced prefix [0, 16 seg0) is one path whose
            // metric and bits the post pass replayed (bit-identical to decoding it here)
            if (seg0 > 0 && P.warm_metric) {
                metric = P.warm_metric[f * PSCL_DL_NSEG + seg0];
                const int lo = 16 * seg0;
                u0 = P.warm_u[2 * f];
                u1 = P.warm_u[2 * f + 1];
                if (lo < 64) {
                    u0 &= (1ULL << lo) - 1ULL;
                    u1 = 0;
                } else {
                    u1 = lo == 64 ? 0ULL : (u1 & ((1ULL << (lo - 64)) - 1ULL));
                }
            }
        }
        uint32_t lastbit = 0;       // the bit decided at the previous phase
        uint32_t tab = 0;           // LDS slot of depths 3..6 (4 bits each); lanes >= LMAX hold
                                    // a copy of their path's table
        int cnt = 1;                // live paths of this frame (group-uniform)
        int j = 0;                  // info index (wave-uniform)
        bool pre_ok = false;        // Lpre holds the tail of this phase's leaf (wave-uniform)
        bool ordered = true;        // every path's lane is its list position (wave-uniform)
        double Lpre = 0.0;
        // wave masks of lane predicates (ballots of plain compares, ANDed in SGPRs)
        const uint64_t vmask = wmask(fvalid);
        constexpr uint64_t KPATH = group_prefix_mask<G>(LMAX), KGE1 = ~group_prefix_mask<G>(1);
        const uint64_t LMASK = group_prefix_mask<G>(L);
        uint64_t amb = 0;  // APX: lanes that saw an ordering closer than the margin
        // the clamp-free screening tail (pscl_softplus_tail_scr_nc, L >= 4) needs every tree LLR
        // below 2^30 in magnitude, and |tree LLR| <= the sum of the frame's 128 channel
        // magnitudes: each lane sums the magnitudes of the channel LLRs it holds (16 or 8 lanes
        // of a frame cover all 128), and a frame where a lane's sum reaches 2^25 -- or is NaN
        // (the sum propagates it) -- goes to the exact re-decode.  L = 8: the lane's 8 registers
        // here; L = 4: its 16 values at the phase-0 recompute
        constexpr bool kTailNC = APX && PSCL_TAIL_NC && LMAX >= 4;
        if constexpr (kTailNC && Ly::CREG) {
            double cs = fabs(creg[0]);
#pragma unroll
            for (int m = 1; m < 8; ++m) cs = cs + fabs(creg[m]);
            amb = wmask(!(cs < 0x1p25));
        }
        // high words of two metrics (non-negative doubles: the words order like the values):
        // b - a <= margin, a < b not certain
        auto near_or_below = [](uint32_t a, uint32_t b) { return (int32_t)(b - a) <= (int32_t)PSCL_SCR_H; };
        auto hiw = [](double m) { return (uint32_t)(pscl_asu64(m) >> 32); };
        // PSCL_TAIL_ABS: the tail's error is absolute (glibc_softplus.h), so an ordering a < b of
        // two screening metrics is certain when b exceeds a by the absolute margin plus a relative
        // 2^-40 for the fp64 summation: hi(b) > hi(up(a)), up(a) = a (1 + 2^-40) + margin (one fma;
        // the high words of non-negative doubles order like the values)
        auto hiw_up = [&](double m) { return hiw(__builtin_fma(m, 1.0 + 0x1p-40, PSCL_TAIL_ABS_MARGIN)); };

        // phase body, specialised on t = phi mod 16 (the subtree shape of the phase is fixed by
        // t); blk = phi / 16 is a compile-time constant too in the CODE != 0 kernels
        auto phase = [&](const auto blk, auto TC) {
            constexpr int PT = decltype(TC)::value;
            const int phi = (int)blk * 16 + PT;
            const int start = PT ? kn - __builtin_ctz((unsigned)PT) : ((int)blk ? 3 - __builtin_ctz((unsigned)(int)blk) : 1);
            const uint64_t infow = phi < 64 ? info0 : info1;
            const bool is_info = (infow >> (phi & 63)) & 1;
            // info index: a compile-time constant with a compiled-in code (warm starts enter
            // the unrolled phases part way), else the running count
            const int jq = CODE != 0 ? (phi < 64 ? __builtin_popcountll(info0 & ((1ULL << (phi & 63)) - 1ULL))
                                                 : __builtin_popcountll(info0) +
                                                       __builtin_popcountll(info1 & ((1ULL << (phi & 63)) - 1ULL)))
                                     : j;
            if constexpr (kFixedList) {  // min(2^j, L) paths after j information bits
                const int jb = phi < 64 ? __builtin_popcountll(info0 & ((1ULL << (phi & 63)) - 1))
                                        : __builtin_popcountll(info0) + __builtin_popcountll(info1 & ((1ULL << (phi & 63)) - 1));
                cnt = jb >= Ly::LOG_LM ? LMAX : (1 << jb);
            }
            // lanes g < cnt (cnt is group-uniform; a compile-time constant with kFixedList)
            const uint64_t cmask = kFixedList ? group_prefix_mask<G>(cnt) : wmask(g < cnt);
#ifdef PSCL_PHASE_MARKERS  // asm listing analysis only
            asm volatile("; PHASE %0" ::"n"(PT));
#endif
            // ---- depths 1-3 recomputed from the channel (phi % 16 == 0)
            if (start <= 3 && !(PSCL_ABLATE & 12) && !(APX && (PSCL_APX_ABLATE & 2))) {
                const bool r1 = phi >= 64, r2 = (phi >> 5) & 1, r3 = (phi >> 4) & 1;
                // path lanes: partial sums of the left siblings at depths 1, 2, 3
                uint64_t X1 = 0;
                uint32_t X2 = 0, X3 = 0;
                if (r1) X1 = polar_transform64(u0);
                if (r2) {  // u[32(k2-1), 32 k2), k2 = phi >> 5 odd
                    const int lo = phi - (phi & 31) - 32;
                    X2 = polar_transform32((uint32_t)((lo >= 64 ? u1 : u0) >> (lo & 63)));
                }
                if (r3) {  // u[phi-16, phi)
                    const int lo = phi - 16;
                    X3 = polar_transform16((uint32_t)((lo >= 64 ? u1 : u0) >> (lo & 63)) & 0xffffu);
                }
                if (LMAX <= 2 && !CH) {
                    // few lanes per frame: 16-lane jobs, one (frame, path) each, so every
                    // channel load instruction reads whole 128-byte rows of 4 frames
                    const int e = lane & 15, slot = lane >> 4;
#pragma unroll 2
                    for (int it = 0; it < F * LMAX / 4; ++it) {
                        const int job = it * 4 + slot;
                        const int fj = job / LMAX, p = job % LMAX;
                        const int owner = fj * G + p;
                        const double* cj = reinterpret_cast<const double*>(shfl_u64((uint64_t)chan, fj * G));
                        double c[8];
#pragma unroll
                        for (int m = 0; m < 8; ++m) c[m] = cj[e + 16 * m];
                        uint64_t x1 = 0;
                        uint32_t x2 = 0, x3 = 0;
                        if (r1) x1 = shfl_u64(X1, owner);
                        if (r2) x2 = bperm32(X2, owner);
                        if (r3) x3 = bperm32(X3, owner);
                        double d1[4];
#pragma unroll
                        for (int m = 0; m < 4; ++m)
                            d1[m] = r1 ? g_node_wbit(c[m], c[m + 4], (uint32_t)(x1 >> (32 * (m >> 1))), (uint32_t)(e + 16 * (m & 1)))
                                       : f_minsum(c[m], c[m + 4]);
                        double d2[2];
#pragma unroll
                        for (int s2 = 0; s2 < 2; ++s2)
                            d2[s2] = r2 ? g_node(d1[s2], d1[s2 + 2], (x2 >> (e + 16 * s2)) & 1u) : f_minsum(d1[s2], d1[s2 + 2]);
                        const double d3 = r3 ? g_node(d2[0], d2[1], (x3 >> e) & 1u) : f_minsum(d2[0], d2[1]);
                        A[fj * Ly::FSTRIDE + Ly::OFF3 + Ly::at(16, e, p)] = d3;
                    }
                } else
#pragma unroll
                for (int q = 0; q < 16 / G + (G > 16); ++q) {
                    const int e = g + G * q;
                    double c[8];
#pragma unroll
                    for (int m = 0; m < 8; ++m) {
                        if constexpr (CREG) c[m] = creg[m];  // (G == 16: e == g)
                        else c[m] = CH ? Af[e + 16 * m] : chan[e + 16 * m];
                    }
                    if constexpr (kTailNC && !CREG) {  // (the check above, at phase 0)
                        if (phi == 0) {
                            double cs = fabs(c[0]);
#pragma unroll
                            for (int m = 1; m < 8; ++m) cs = cs + fabs(c[m]);
                            amb |= wmask(!(cs < 0x1p24));  // (two such sums per lane at G = 8)
                        }
                    }
                    double d1l[4];
#pragma unroll
                    for (int m = 0; m < 4; ++m) d1l[m] = r1 ? 0.0 : f_minsum(c[m], c[m + 4]);  // (r1: g nodes below)
                    // each path lane publishes its partial sums once; every lane then reads those of
                    // the path it works on (one ds_read_b128 instead of four ds_bpermute)
                    uint4* xs_lds = reinterpret_cast<uint4*>(Af + Ly::OFFX);
                    if (q == 0 && (r1 || r2 || r3)) {
                        // (X2 beside X2 >> 16 | X3 << 16: one 64-bit shift brings bits e and e + 16 of X2
                        // to bit 31 of the two halves -- scl128_lane.hip's recompute)
                        if (path_lane) xs_lds[g] = make_uint4((uint32_t)X1, (uint32_t)(X1 >> 32), X2, (X2 >> 16) | (X3 << 16));
                        wave_lds_fence();
                    }
                    // left-left quarter (phi = 0, 16): depth 2 = f(depth 1) is the same for every path
                    const bool shared2 = !r1 && !r2;
                    double d2s[2];
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) d2s[s2] = shared2 ? f_minsum(d1l[s2], d1l[s2 + 2]) : 0.0;
                    // paths that exist (compiled-in codes know: phi = 0 has one)
                    const int npaths = kFixedList && cnt < LMAX ? cnt : LMAX;
#pragma unroll
                    for (int p0 = 0; p0 < LMAX; ++p0) {
                        if (p0 >= npaths) break;
                        // lane e takes path (p0 + e) mod LMAX in step p0: the 16 lanes of a frame
                        // then store to 16 distinct bank pairs (the same path for every lane put
                        // the 16 stores on 2 bank pairs: 8-way conflicts)
                        const int p = npaths == LMAX ? (p0 + e) & (LMAX - 1) : p0;
                        uint64_t x1 = 0, x23 = 0;
                        if (r1 || r2 || r3) {
                            const uint4 xv = xs_lds[p];
                            x1 = ((uint64_t)xv.y << 32) | xv.x;
                            x23 = ((uint64_t)xv.w << 32) | xv.z;
                        }
                        // the g nodes' bits at bit 31 of a half of a 64-bit shift (two nodes per shift)
                        const uint64_t s1[2] = {r1 ? x1 << (31u - (uint32_t)e) : 0ULL, r1 ? x1 << (15u - (uint32_t)e) : 0ULL};
                        const uint64_t s2w = r2 ? x23 << (31u - (uint32_t)e) : 0ULL;
                        double d1[4];
#pragma unroll
                        for (int m = 0; m < 4; ++m)
                            d1[m] = r1 ? g_node_bit31(c[m], c[m + 4], (uint32_t)(s1[m & 1] >> (32 * (m >> 1)))) : d1l[m];
                        double d2[2];
#pragma unroll
                        for (int s2 = 0; s2 < 2; ++s2)
                            d2[s2] = shared2 ? d2s[s2]
                                     : (r2 ? g_node_bit31(d1[s2], d1[s2 + 2], (uint32_t)(s2w >> (32 * s2))) : f_minsum(d1[s2], d1[s2 + 2]));
                        const double d3 = r3 ? g_node_wbit(d2[0], d2[1], (uint32_t)(x23 >> 32), (uint32_t)e + 16u) : f_minsum(d2[0], d2[1]);
                        Af[Ly::OFF3 + Ly::at(16, e, p)] = d3;
                    }
                }
                wave_lds_fence();
            }
            // ---- depths 4..6 (partial sums of the g node's left sibling: xs, <= 8 bits)
            uint32_t xs = 0;
            if (phi && start >= 4 && start <= 6) {  // u[phi-w, phi), w = 8, 4, 2
                const int w = 1 << (kn - start), lo = phi - w;
                xs = polar_transform8((uint32_t)((lo >= 64 ? u1 : u0) >> (lo & 63)) & ((1u << w) - 1u));
            }
            if (!(PSCL_ABLATE & 4) && !(APX && (PSCL_APX_ABLATE & 4)) && start <= 6) {
                // (DPP evaluated by every lane first: inside ?: only the selected lanes would
                // run it, and a DPP that reads an inactive lane gets 0)
                const uint32_t tabp = tab;
                const double* lb = Af + 2 * g;
                const uint32_t xsp = merge_from_lower<G, LMAX>(xs, xs, lane);
                if (start <= 4) step_depth<LMAX, CH, 4>(Af, lb, g, tabp, xsp, start == 4, start == 4 && phi);
                if (start <= 5) step_depth<LMAX, CH, 5>(Af, lb, g, tabp, xsp, start == 5, start == 5);
                if (start <= 6) step_depth<LMAX, CH, 6>(Af, lb, g, tabp, xsp, start == 6, start == 6);
            }
            if (start <= 6) {  // this path's own slot at every depth rewritten this phase
                // (same update in the upper lane's copy: cpath is the path of both lanes)
                const int s0 = start < 3 ? 3 : start;
                const uint32_t mask = (0xffffu << (4 * (s0 - 3))) & 0xffffu;
                tab = (tab & ~mask) | ((uint32_t)cpath * 0x1111u & mask);
            }
            // ---- leaf LLRs.  Lanes >= LMAX: the sibling leaf (phi+1) given bit 0 here.
            // (depth 6 was just rewritten into the path's own slot at even phases)
            const double2 lab = reinterpret_cast<const double2*>(Af + Ly::OFF6)[start <= 6 ? cpath : slot_at(tab, 6)];
            const double la = lab.x, lb = lab.y;
            const uint32_t xleaf = lastbit;  // u[phi - 1], the left sibling's bit at odd phases
            // Upper lanes: the next (odd) leaf given this phase's bit -- bit 0 at frozen phases;
            // at even information phases of the screening decode, the better child's bit (the
            // sign of this leaf), which every path keeps whenever the list update below takes
            // its keep-the-better-children path
#if PSCL_LEAF_BLEND
            // branch-free: every lane evaluates both forms and keeps its own by a bit blend (a
            // ternary on path_lane around the f asm becomes a divergent branch)
            double lam;
            if (phi & 1) {  // path lanes g(u[phi-1]), upper lanes g(0): one g with a per-lane bit
                lam = g_node(la, lb, path_lane ? xleaf : 0u);
            } else {
                const double fv = f_minsum(la, lb);
                const double up = (APX && is_info) ? g_node(la, lb, sign_bit(fv)) : lb + la;
                const uint64_t m = path_lane ? ~0ULL : 0ULL;
                lam = pscl_asf64((pscl_asu64(fv) & m) | (pscl_asu64(up) & ~m));
            }
            if (PSCL_ABLATE & 128) lam = la;
#else
            double lam_up = lb + la;
            if (APX && is_info && !(phi & 1)) lam_up = g_node(la, lb, sign_bit(f_minsum(la, lb)));
            const double lam = (PSCL_ABLATE & 128) ? la : (path_lane ? ((phi & 1) ? g_node(la, lb, xleaf) : f_minsum(la, lb)) : lam_up);
#endif
            // ---- metric tail log1p(exp(-|llr|)) (scl.py:102-105)
            double Lt;
            const uint64_t lpre_up = from_upper_half64<G, LMAX>(pscl_asu64(Lpre), lane);
            if (pre_ok) {
                Lt = pscl_asf64(lpre_up);
            } else {
                Lt = (PSCL_ABLATE & 1) ? lam * 0.5
                     : (APX ? ((PSCL_APX_ABLATE & 1) ? fabs(lam) * 0x1p-20
                                                       : (PSCL_TAIL_ABS ? pscl_softplus_tail_abs(lam)
                                                          : (kTailNC ? pscl_softplus_tail_scr_nc(lam) : pscl_softplus_tail_scr(lam))))
                            : pscl_softplus_tail_bf(lam, T));
            }
            const bool frozen_even = !is_info && !(phi & 1);
            Lpre = Lt;
            pre_ok = frozen_even;
            // children metrics (scl.py:102-105): the child along the LLR sign pays Lt, the
            // other |lam| + Lt; an exactly zero LLR gives both LOGE2 (rare wave branch)
            const bool neg = lam < 0.0;
            const double mgd = metric + Lt, mbd = metric + (fabs(lam) + Lt);

            if constexpr (APX) {
                // Screening: with every ordering decision beyond the margin, the stable sort's
                // tie keys never act, so the list order in between does not matter -- only which
                // children survive a full list (the boundary between the L-th and (L+1)-th
                // smallest metric) and, at the end, the final order.  Paths stay in lanes
                // 0..cnt-1 in any order; frozen phases only advance the metrics.  An exactly
                // zero LLR needs no special case: both children get metric + tail(0) (= the
                // exact LOGE2 within the tail's bound), a tie the margin tests catch.
                if (!is_info) {  // bit 0: metric + max(-lam, 0) + tail (any rounding order will do)
                    metric = metric + (relu_neg(lam) + Lt);
                    lastbit = 0;
                    return;
                }
                // better / worse child (any rounding order will do here)
                const double mg = metric + Lt, mb = mg + fabs(lam);
                const double m0 = neg ? mb : mg, m1 = neg ? mg : mb;  // bit-0 / bit-1 child
                int ncnt = 2 * cnt < L ? 2 * cnt : L;
                int src;
                uint32_t b;
                uint64_t nm;
                // forced bits (FS: the DL-SCL retry decodes, scl.py:146-161): a force vector
                // fixes a prefix of the information bits, so a forced frame holds one path and
                // takes the forced child -- no ordering decision (frames of a wavefront may be
                // forced or free at a phase: cnt and the branches below are per frame)
                bool forced_here = false;
                uint32_t fbit = 0;
                if constexpr (FS) {
                    if (force) {
                        forced_here = (((jq < 64 ? fm0 : fm1) >> (jq & 63)) & 1) != 0;
                        fbit = (uint32_t)(((jq < 64 ? fv0 : fv1) >> (jq & 63)) & 1);
                    }
                }
                if (FS && forced_here) {
                    src = lane;
                    b = fbit;
                    nm = pscl_asu64(b ? m1 : m0);
                    ncnt = cnt;
                } else if (2 * cnt <= L) {
                    // every child survives: bit 0 stays in lane p, bit 1 goes to lane cnt + p
                    src = gbase + (g & (cnt - 1));
                    b = (g & cnt) ? 1u : 0u;
                    const uint64_t pm1 = shfl_u64(pscl_asu64(m1), src);
                    nm = b ? pm1 : pscl_asu64(m0);
                } else {
                    // full list: the better children survive when every worse child exceeds the
                    // largest better child by the margin (group max of the high words over
                    // duplicated keys)
                    const uint32_t kx = PSCL_TAIL_ABS ? hiw_up(mg) : hiw(mg);
                    uint32_t mx = merge_from_lower<G, LMAX>(kx, kx, lane);
                    static_for<Ly::LOG_LM>([&](auto SC) {
                        constexpr int S = 1 << decltype(SC)::value;
                        const uint32_t o = grot32c<G, S>(mx, lane);
                        mx = o > mx ? o : mx;
                    });
                    const uint64_t badm = wmask(PSCL_TAIL_ABS ? hiw(mb) <= mx : near_or_below(mx, hiw(mb)));
#ifdef PSCL_STATS  // screening full-list info phases by the wave's worst frame: worse children
                   // within the margin of the largest better child (0, 1, 2, >= 3) -> slots 12..15
                    if (lane == 0 && P.counters) {
                        int worst = 0;
                        for (int fr = 0; fr < F; ++fr) {
                            const int pc = __builtin_popcountll((badm & vmask & KPATH) >> (fr * G) & ((1ULL << LMAX) - 1));
                            worst = pc > worst ? pc : worst;
                        }
                        atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + 12 + (worst < 3 ? worst : 3), 1ULL);
                    }
#endif
                    if (!(PSCL_APX_ABLATE & 32) && ((PSCL_APX_ABLATE & 8) || (badm & vmask & KPATH) == 0)) {
                        // (lam != +-0 here: a zero LLR gives mbd == mgd, never clear of the margin,
                        // so the sign bit is the better child's bit)
                        const uint32_t gb = sign_bit(lam);
                        metric = mg;
                        lastbit = gb;
                        if (phi < 64) u0 |= (uint64_t)gb << phi; else u1 |= (uint64_t)gb << (phi - 64);
                        ++j;
                        // the upper lanes' tail is the next leaf's (see lam_up); not with forced
                        // bits, where the frames of a wavefront may take other branches here
                        pre_ok = !FS && !(phi & 1);
                        return;
                    }
                    // rank the 2L children on the high words; lane r takes the child ranked r.
                    // Each position 0..L claimed exactly once and the L-th / (L+1)-th smallest
                    // apart by the margin certify the survivor set (ties leave a position unclaimed).
                    const uint64_t km = merge_from_lower64<G, LMAX>(pscl_asu64(m0), pscl_asu64(m1), lane);
                    uint32_t r = 0;
                    rank_step_h<G, 1, G>((uint32_t)(km >> 32), lane, r);
                    const int c = __builtin_amdgcn_ds_permute((gbase + (int)(r & (G - 1))) << 2, g) & (G - 1);
                    const uint32_t rr = bperm32(r, gbase + c);
                    nm = shfl_u64(km, gbase + c);
                    const uint64_t claim = group_prefix_mask<G>(L + 1);
                    const uint64_t bnd = claim & ~group_prefix_mask<G>(L);
                    const uint32_t nmh = (uint32_t)(nm >> 32);
                    const bool bnear = PSCL_TAIL_ABS ? nmh <= prev_lane32(hiw_up(pscl_asf64(nm))) : near_or_below(prev_lane32(nmh), nmh);
                    amb |= ((wmask(rr != (uint32_t)g) & claim) | (wmask(bnear) & bnd)) & vmask;
#ifdef PSCL_DEBUG_AMB
                    {
                        const uint64_t cm = wmask(rr != (uint32_t)g) & claim & vmask, bm = wmask(near_or_below(prev_lane32(nmh), nmh)) & bnd & vmask;
                        if (f0 == 0 && lane < 16 && (cm | bm)) printf("phi %d lane %d r %u c %d rr %u nmh %08x prev %08x claimfail %d bndfail %d\n", phi, lane, r, c, rr, nmh, prev_lane32(nmh), (int)((cm >> lane) & 1), (int)((bm >> lane) & 1));
                    }
#endif
                    src = gbase + (c & (LMAX - 1));
                    b = c >= LMAX ? 1u : 0u;
                }
                metric = pscl_asf64(nm);
                u0 = shfl_u64(u0, src);
                if (phi >= 64) u1 = shfl_u64(u1, src);
                const uint32_t ntab = bperm32(tab, src);
                tab = merge_from_lower<G, LMAX>(ntab, ntab, lane);
                if (phi < 64) u0 |= (uint64_t)b << phi; else u1 |= (uint64_t)b << (phi - 64);
                lastbit = b;
                cnt = ncnt;
                ++j;
                return;
            }

            if (!is_info) {
                // frozen: bit 0, metrics advance, stable re-rank in place (lanes do not move).
                // While lane order is list order, the stable sort is the identity exactly when
                // the new metrics stay non-decreasing along the lanes: one adjacent compare.
                double m0 = neg ? mbd : mgd;
                if (PSCL_RARE(lam == 0.0)) m0 = lam == 0.0 ? metric + PSCL_LOGE2 : m0;
                metric = m0;
                lastbit = 0;
                bool moved = true;
                if (ordered && !(PSCL_ABLATE & 256)) {
                    const uint64_t pv = prev_lane64(pscl_asu64(m0));
                    moved = (wmask(pv > pscl_asu64(m0)) & vmask & KPATH & KGE1 & cmask) != 0;
                }
#ifdef PSCL_STATS  // diagnostic build (tools/fastpath_stats.py): counters[8..11] of a 16-slot buffer
                if (lane == 0 && P.counters) {
                    atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + 8, 1ULL);
                    if (!moved) atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + 9, 1ULL);
                }
#endif
                if (!moved) return;
                // (a full list needs no empty-slot keys: the upper lanes are overwritten next)
                const bool kv = (kFixedList && cnt == LMAX) || g < cnt;
                uint64_t km = kv ? pscl_asu64(m0) : 0x7ff0000000000000ULL;
                uint32_t kt = kv ? rank : 0x7fffffffu;
                // duplicate the path keys into the upper half: LMAX-1 rotations then see every path
                km = merge_from_lower64<G, LMAX>(km, km, lane);
                kt = merge_from_lower<G, LMAX>(kt, kt, lane);
                uint32_t r = 0;
                if (!(PSCL_ABLATE & 18)) rank_step_n<G, 1, LMAX>((uint32_t)(km >> 32), (uint32_t)km, kt, lane, r);
                if (path_lane) rank = r;
                ordered = (wmask(rank != (uint32_t)g) & vmask & KPATH & cmask) == 0;
            } else {
                // info, full list, lane order = list order: when every path's worse child
                // (against the LLR sign) is strictly worse than every better child and the
                // better children keep the lane order, the survivors are the better children
                // in place -- the outcome of the stable sort, with no ranking and no moves
                if (ordered && !sc_hard && !(PSCL_ABLATE & 256)) {
                    const uint32_t gb = neg ? 1u : 0u;
                    const uint64_t mg = pscl_asu64(mgd), mb = pscl_asu64(mbd);
                    const uint64_t pv = prev_lane64(mg);
                    const uint64_t top = shfl_u64(mg, gbase + L - 1);
                    bool forced_here = false;
                    if (FS && force) forced_here = (((jq < 64 ? fm0 : fm1) >> (jq & 63)) & 1) != 0;
                    uint64_t badm = wmask(lam == 0.0) | (wmask(pv > mg) & KGE1) | wmask(mb <= top);
                    if (FS && force) badm |= wmask(forced_here);
                    if (kFixedList) {
                        if (cnt != L) badm = ~0ULL;
                    } else {
                        badm |= wmask(cnt != L);
                    }
                    if ((badm & vmask & KPATH & LMASK) == 0) {
                        if (HIST && path_lane && g < L) {
                            hist_llr[jq * L + g] = lam;
                            hist_par[jq * L + g] = (uint8_t)g;
                        }
                        metric = pscl_asf64(mg);
                        lastbit = gb;
                        if (gb) {
                            if (phi < 64) u0 |= 1ULL << phi; else u1 |= 1ULL << (phi - 64);
                        }
                        ++j;
#ifdef PSCL_STATS
                        if (lane == 0 && P.counters) atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + 11, 1ULL);
#endif
                        return;
                    }
                }
#ifdef PSCL_STATS
                if (lane == 0 && P.counters) atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + 10, 1ULL);
#endif
                // info: children (bit 0 in lane g, bit 1 in lane g + LMAX) of every path
                double m0 = neg ? mbd : mgd, m1 = neg ? mgd : mbd;
                if (PSCL_RARE(lam == 0.0)) {
                    m0 = lam == 0.0 ? metric + PSCL_LOGE2 : m0;
                    m1 = lam == 0.0 ? metric + PSCL_LOGE2 : m1;
                }
                // bit-0 child in lane g, bit-1 child (from lane g - LMAX) in lane g + LMAX
                uint64_t km = merge_from_lower64<G, LMAX>(pscl_asu64(m0), pscl_asu64(m1), lane);
                const uint32_t myrank = merge_from_lower<G, LMAX>(rank, rank, lane);
                bool kval = cpath < cnt;
                int ncnt = 2 * cnt < L ? 2 * cnt : L;  // both children (scl.py:163-168)
                if (FS && sc_hard) {                  // sc_decode polar.py:149-153
                    const double plam = pscl_asf64(from_lower_half64<G, LMAX>(pscl_asu64(lam), lane));
                    kval = kval && cbit == (uint32_t)((cbit ? plam : lam) < 0.0);
                    ncnt = cnt;
                } else if (FS && force) {             // forced bits (scl.py:146-161), per frame
                    const uint64_t fmw = jq < 64 ? fm0 : fm1, fvw = jq < 64 ? fv0 : fv1;
                    if ((fmw >> (jq & 63)) & 1) {
                        kval = kval && cbit == (uint32_t)((fvw >> (jq & 63)) & 1);
                        ncnt = cnt;
                    }
                }
                if (!kval) km = 0x7ff0000000000000ULL;
                const uint32_t kt = kval ? 2u * myrank + cbit : 0x7fffffffu;
                uint32_t r = 0;
                int c;
#if PSCL_RANK_M
                // rank on the metric alone, then check that the ranks 0..ncnt are all claimed
                // (lane g pulls the rank of the lane it received); equal metrics among the
                // candidates that matter leave a hole and take the full (metric, 2*rank + bit) key
                rank_step_m<G, 1, G>((uint32_t)(km >> 32), (uint32_t)km, lane, r);
                c = __builtin_amdgcn_ds_permute((gbase + (int)(r & (G - 1))) << 2, g);
                {
                    const uint32_t rr = bperm32(r, gbase + (c & (G - 1)));
                    const uint64_t chk = kFixedList ? group_prefix_mask<G>(ncnt + 1) : wmask(g <= ncnt);
                    if (__builtin_expect((wmask(rr != (uint32_t)g) & chk) != 0, 0)) {
                        r = 0;
                        rank_step<G, 1>((uint32_t)(km >> 32), (uint32_t)km, kt, lane, r);
                        c = __builtin_amdgcn_ds_permute((gbase + (int)(r & (G - 1))) << 2, g);
                    }
                }
#else
                if (!(PSCL_ABLATE & 2)) rank_step<G, 1>((uint32_t)(km >> 32), (uint32_t)km, kt, lane, r);
                else r = kt & 15u;
                // survivor with list position r -> lane r of the group (push), scl.py:174
                c = (PSCL_ABLATE & 32) ? g : __builtin_amdgcn_ds_permute((gbase + (int)(r & (G - 1))) << 2, g);
#endif
                const int cc = (g < ncnt) ? c : g;
                const int par_g = cc & (LMAX - 1);
                const uint32_t b = cc >= LMAX ? 1u : 0u;
                const int ps2 = gbase + par_g;
                const uint64_t nm = (PSCL_ABLATE & 32) ? km : shfl_u64(km, gbase + cc);
                const uint64_t nu0 = (PSCL_ABLATE & 32) ? u0 : shfl_u64(u0, ps2);
                const uint64_t nu1 = (PSCL_ABLATE & 32) || phi < 64 ? u1 : shfl_u64(u1, ps2);  // u1 = 0 before 64
                const uint32_t ntab = (PSCL_ABLATE & 32) ? tab : bperm32(tab, ps2);
                if (HIST) {
                    const uint64_t plam_h = shfl_u64(pscl_asu64(lam), ps2);
                    if (g < ncnt && path_lane) {
                        hist_llr[jq * L + g] = pscl_asf64(plam_h);  // decision LLR (scl.py:158,166)
                        hist_par[jq * L + g] = (uint8_t)par_g;
                    }
                }
                metric = pscl_asf64(nm);
                u0 = nu0;
                u1 = nu1;
                // the upper lanes copy their (new) path's table
                tab = merge_from_lower<G, LMAX>(ntab, ntab, lane);
                if (b) {
                    if (phi < 64) u0 |= 1ULL << phi; else u1 |= 1ULL << (phi - 64);
                }
                lastbit = b;
                rank = (uint32_t)g;
                cnt = ncnt;
                ordered = true;
                ++j;
            }
        };
        // all 128 phases unrolled with phi a compile-time constant (with CODE != 0 the
        // information set is too: every frozen/info branch and the info index fold away)
        if constexpr (CODE != 0 && FS) {
            // forced decodes enter at their warm-start segment (seg0 = 0 without one)
            auto seg = [&](auto SB) { static_for<16>([&](auto TC) { phase(SB, TC); }); };
            using std::integral_constant;
            switch (seg0) {
                case 0: seg(integral_constant<int, 0>{}); [[fallthrough]];
                case 1: seg(integral_constant<int, 1>{}); [[fallthrough]];
                case 2: seg(integral_constant<int, 2>{}); [[fallthrough]];
                case 3: seg(integral_constant<int, 3>{}); [[fallthrough]];
                case 4: seg(integral_constant<int, 4>{}); [[fallthrough]];
                case 5: seg(integral_constant<int, 5>{}); [[fallthrough]];
                case 6: seg(integral_constant<int, 6>{}); [[fallthrough]];
                default: seg(integral_constant<int, 7>{});
            }
        } else if constexpr (CODE != 0) {
            static_for<kN>([&](auto PC) { phase(std::integral_constant<int, (decltype(PC)::value >> 4)>{}, std::integral_constant<int, (decltype(PC)::value & 15)>{}); });
        } else {
            for (int blk = 0; blk < kN / 16; ++blk)
                static_for<16>([&](auto TC) { phase(blk, TC); });
        }

        // ---- epilogue: u[info_set] and its CRC syndrome, best = lowest-ranked CRC pass
        // (LDS tables: u-byte gather, then ib-nibble syndrome)
        uint64_t ib0 = 0, ib1 = 0;
        uint32_t syn = 0;
        if (!(PSCL_ABLATE & 64)) {
            int off = 0;  // information bits below byte k (wave-uniform)
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t byte = (uint32_t)(((k < 8 ? u0 : u1) >> (8 * (k & 7))) & 255u);
                const uint64_t c = GT[k * 256 + byte];
                if (off < 64) {
                    ib0 |= c << off;
                    if (off > 56) ib1 |= c >> (64 - off);
                } else {
                    ib1 |= c << (off - 64);
                }
                off += __builtin_popcount((uint32_t)(((k < 8 ? info0 : info1) >> (8 * (k & 7))) & 255u));
            }
            if (P.has_crc) {
                const int k4 = (K + 3) >> 2;
                const int m0 = k4 < 16 ? k4 : 16;
                for (int m = 0; m < m0; ++m) syn ^= ST[m * 16 + (uint32_t)((ib0 >> (4 * m)) & 15u)];
                for (int m = 16; m < k4; ++m) syn ^= ST[m * 16 + (uint32_t)((ib1 >> (4 * (m - 16))) & 15u)];
            }
        }
        if constexpr (APX && !(PSCL_APX_ABLATE & 16)) {
            // the final list order (best = first CRC pass, and its index): rank on the metric,
            // certified by every position 0..cnt-1 claimed once and sorted neighbours apart by
            // the margin.  Upper lanes hold copies, rank among the same keys and push into the
            // upper half.
            uint32_t kh = g < cnt ? hiw(metric) : 0x7ff00000u;
            kh = merge_from_lower<G, LMAX>(kh, kh, lane);
            uint32_t r = 0;
            rank_step_h<G, 1, LMAX>(kh, lane, r);
            const int c = __builtin_amdgcn_ds_permute((gbase + (g & LMAX) + (int)(r & (LMAX - 1))) << 2, g) & (G - 1);
            const uint32_t rr = bperm32(r, gbase + c);
            const uint32_t nh = bperm32(kh, gbase + c);
            bool fnear;
            if constexpr (PSCL_TAIL_ABS) {
                uint32_t ku = g < cnt ? hiw_up(metric) : 0x7ff00000u;
                ku = merge_from_lower<G, LMAX>(ku, ku, lane);
                fnear = nh <= prev_lane32(bperm32(ku, gbase + c));
            } else {
                fnear = near_or_below(prev_lane32(nh), nh);
            }
            const uint64_t live = kFixedList ? group_prefix_mask<G>(cnt) : wmask(g < cnt);
            amb |= ((wmask(rr != (uint32_t)g) & live) | (wmask(fnear) & live & KGE1)) & vmask;
#ifdef PSCL_DEBUG_AMB
            if (f0 == 0 && lane < 16) printf("final lane %d r %u c %d rr %u kh %08x nh %08x prev %08x\n", lane, r, c, rr, kh, nh, prev_lane32(nh));
#endif
            rank = r;
        }
        // APX: a frame with an uncertain ordering is handed to the exact re-decode
        const bool famb = APX && ((amb >> gbase) & (G == 64 ? ~0ULL : ((1ULL << (G & 63)) - 1))) != 0;
        if (APX && !PSCL_APX_ABLATE && famb && g == 0 && fvalid) {
            if (FS && P.amb_elist) {  // DL-SCL retry round: into the entry's bucket, flagged deferred
                const int fseg = P.warm_apx ? 0 : pscl_bucket_of(fsafe, bpre);  // (screening warm metrics: exact from phase 0)
                const int slot = atomicAdd(P.amb_count + fseg * PSCL_DL_CSTRIDE, 1);
                P.amb_elist[(int64_t)fseg * P.bcap + slot] = (int32_t)f;
                P.flags[f] = PSCL_DL_DEFERRED;
            } else {
                P.amb_list[atomicAdd(P.amb_count, 1)] = f;
            }
        }
        const bool active = path_lane && g < cnt && fvalid && !famb;
        const int64_t fo = P.out_by_row ? frow : f;  // output row
        uint32_t pm = (active && syn == 0) ? (1u << rank) : 0u;
        pm = or_reduce_group<G>(pm, lane);
        const int best = (P.has_crc && pm) ? __builtin_ctz(pm) : 0;
        if (active) {
            const int64_t row = fo * L + rank;
            if (P.metrics) P.metrics[row] = metric;
            if (P.cands) {
                P.cands[row * PW] = ib0;
                if (PW > 1) P.cands[row * PW + 1] = ib1;
            }
            if (HIST && P.info_llrs) {
                int cur = g;
                for (int jj = K - 1; jj >= 0; --jj) {
                    P.info_llrs[row * K + jj] = hist_llr[jj * L + cur];
                    cur = hist_par[jj * L + cur];
                }
            }
            if ((int)rank == best) {
                const bool bpass = P.has_crc ? (syn == 0) : true;
                if (HIST && P.best_info_llrs) {
                    int cur = g;
                    for (int jj = K - 1; jj >= 0; --jj) {
                        P.best_info_llrs[fo * K + jj] = hist_llr[jj * L + cur];
                        cur = hist_par[jj * L + cur];
                    }
                }
                if (P.best) {
                    P.best[fo * PW] = ib0;
                    if (PW > 1) P.best[fo * PW + 1] = ib1;
                }
                if (P.flags) P.flags[fo] = (uint8_t)((bpass ? PSCL_FLAG_CRC_PASS : 0u) | (uint32_t)best);
                if (P.n_paths) P.n_paths[fo] = cnt;
                if (P.ref && !(APX && PSCL_APX_ABLATE)) {  // (ablation timings: wrong frames, no counts)
                    if constexpr (HIST && !PSCL_HIST_AGG) {
                        // (the history instances keep per-frame atomics: their register budget is
                        // spent -- four more live counters spill further, and the rate-matched L = 8
                        // history instance then measured wrong decision LLRs; see docs/HISTORY.md §5.6)
                        count_errors(P.counters, ib0, ib1, P.ref[fo * PW], PW > 1 ? P.ref[fo * PW + 1] : 0, P.k_payload,
                                     bpass);
                    } else {
                        const uint64_t ibw[2] = {ib0, ib1};
                        tally_errors(ibw, P.ref + fo * PW, PW, P.k_payload, bpass, cfe, cbe, cpe, cpb);
                    }
                }
            }
        }
        wave_lds_fence();
    }
    if constexpr (!HIST || PSCL_HIST_AGG)
        if (P.ref) flush_counts_p(P, (int64_t)blockIdx.x * wpg + wave, cfe, cbe, cpe, cpb);
    if (P.ref && !P.out_by_row && blockIdx.x == 0 && threadIdx.x == 0)
        atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + PSCL_CNT_FRAMES, (unsigned long long)P.B);
}

}  // namespace

#endif
