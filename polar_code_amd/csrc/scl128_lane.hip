// scl128_lane.hip -- the lane-per-path screening decoder for N = 128, L = 8 (the headline decode,
// BASELINE.json: P(128,64)+CRC-24 SCL L = 8) and its launch.
//
// Same contract as the screening pass of scl128_kernel (scl128_impl.h, APX = true; DESIGN.md
// §5.1a): a plain decode of the compiled-in (128,64) code whose path metrics carry the
// bounded-error tail (pscl_softplus_tail_abs); every ordering decision it makes must clear the
// absolute margin, and a frame with an uncertain one is appended to P.amb_list for the exact
// re-decode (the exact kernel, launched by capi.cpp).  Results are therefore bit-identical to
// decode_scl (dl_scl_polar/polar/scl.py:108-209).
//
// Mapping (the difference from scl128_kernel): ONE lane per list path, G = L = 8 lanes per frame,
// F = 8 frames per wavefront.  scl128_kernel gives each frame 2L = 16 lanes, the upper half
// holding the bit-1 children; every per-path step (leaf, tail, metric, list bookkeeping) then runs
// on half-used lanes.  Here a lane holds both children of its path during an information phase:
//   * frozen phase: leaf, tail, metric advance (no ordering decision);
//   * information phase, list growing (its first log2 L): every child survives, bit-1 children
//     move to lanes cnt..2cnt-1;
//   * information phase, full list: if every worse child clears the largest better child by the
//     margin (one DPP max over the frame's 8 lanes) the better children stay in place (the
//     common case); else the 2L children are ranked (each lane counts the keys below its two
//     children: 7 lane permutations -- quad_perm xor 1..3 and the half-row mirror composed with
//     them -- of DPP-fused subtract + add-with-carry), the survivor set is certified (exactly L
//     survivors, the largest survivor's margin-raised key below the smallest non-survivor's key)
//     and each freed lane pulls the j-th surviving worse child of its frame (j-th set bit of an
//     8-bit mask, computed in VALU) with ds_bpermute;
//   * depths 1-3 recomputed every 16 phases from the frame's 128 channel LLRs, which the 8 lanes
//     hold in registers (16 each); depths 3-4 in LDS slots with lazy copies (slot tables), as
//     scl128_kernel, depths 5-6 in the path's registers (PSCL_LANE_REG56, below).
// LDS per frame: depths 3..4 = 24 L doubles (+ pad to the frame stride), the left-sibling partial
// sums of the depth-1..3 recompute aliased onto depth 4; 13 KB per wavefront at L = 8, 12
// wavefronts per CU.  One wavefront per workgroup (no barriers); the epilogue's u-byte gather and
// CRC syndrome tables are read from global memory (L1/L2-resident).  Metrics in bits
// (PSCL_LANE_BITS, scl_lane.h): the channel LLRs scaled by log2 e as they are loaded.
// L = 8 lane map (1): frame = the outer or the inner two quads of a 16-lane row (lanes {0-3, 12-15}
// and {4-11} of row 0, ...), p = lane % 4 + 4 (quad % 2); else frames of 8 consecutive lanes.  A
// ds_read_b128 lane group ({0-3, 12-15, 20-27}, MI355X_MICROARCH.md) then holds exactly two frames,
// one per 128-byte bank half (frame stride = 16 mod 32 doubles), so a frame's data-dependent slot
// reads (any 8 of its 8 slots, 16 B each) never meet another frame's: no LDS bank conflicts by
// construction (8 consecutive lanes put four frames in a group, two per half, whose parent-slot
// reads met: 11.8-16.5 % conflict cycles).  The within-frame permutations are unchanged in p (quad
// perms on p % 4, the mirror p <-> 7 - p).  Measured (profiles/r05k_remap_ab.txt): conflicts 16.5 ->
// 10.7 % of LDS cycles, but the split frame bits cost 212 VALU per wavefront more and the launch
// 1.96-1.97 ms against 1.92-1.95: off by default.
#ifndef PSCL_LANE_REMAP
#define PSCL_LANE_REMAP 0
#endif
#if PSCL_LANE_REMAP
#define PSCL_LANE_FRAME_MIRROR 0x140
#endif
#include "scl_lane.h"

namespace {

// depths 5 and 6 (4 + 2 values per path) in the registers of the path's lane, carried along when a
// lane takes another path's child (1), or in LDS slots with lazy copies like depths 3 and 4 (0):
// LDS per frame 24 L doubles (+ pad) instead of 30 L, 12 wavefronts per CU instead of 10 at L = 8
#ifndef PSCL_LANE_REG56
#define PSCL_LANE_REG56 1
#endif

// frame stride residues (doubles mod 32; see FSTRIDE below): L = 8 8 (stride 200), L = 4 24 (120)
#ifndef PSCL_LANE_FRES8
#define PSCL_LANE_FRES8 8
#endif
#ifndef PSCL_LANE_FRES4
#define PSCL_LANE_FRES4 24
#endif

template <int LMAX>
struct LaneLayout {
    static constexpr int G = LMAX;
    static constexpr int F = 64 / G;
    static constexpr int LOG_G = __builtin_ctz(G);
    static constexpr int OFF3 = 0;              // [8][L][2]
    static constexpr int OFF4 = OFF3 + 16 * LMAX;  // [4][L][2]
    static constexpr int OFF5 = OFF4 + 8 * LMAX;   // [2][L][2] (PSCL_LANE_REG56 = 0)
    static constexpr int OFF6 = OFF5 + 4 * LMAX;   // [1][L][2] (PSCL_LANE_REG56 = 0)
    // the depth-1..3 recompute's partial sums (16 B per path): on depth 6, or on depth 4 when depths
    // 5 and 6 live in registers (depth 4 is rewritten after the recompute has read them)
    static constexpr int OFFX = PSCL_LANE_REG56 ? OFF4 : OFF6;
    static constexpr int RAW = PSCL_LANE_REG56 ? OFF5 : OFF6 + 2 * LMAX;
    // frame stride in doubles: = 8 (mod 32) at L = 8 (200 with REG56; round 6): frames start at
    // 64-byte steps of the 256-byte bank row.  The = 16 stride (208: frames alternate the two
    // 128-byte halves, so a ds_read_b128 lane group's four frames pair up per half) measured 15.6 %
    // LDS bank conflicts against 29 % here, yet the launch is 3-4 % slower (profiles/
    // r06an_frame_stride_ab.txt: strides 192 196 200 204 208 timed) -- the conflict counter is not
    // what bounds this kernel.  = 24 (mod 32) at L = 4 (120; 112 = 16 mod 32 measured 46 % bank
    // conflicts against 4.5 %: the L = 4 kernel's occupancy is bound by its VGPRs, not its LDS)
    static constexpr int FRES = LMAX == 8 ? PSCL_LANE_FRES8 : PSCL_LANE_FRES4;
    static constexpr int FSTRIDE = RAW + (((FRES - RAW) % 32) + 32) % 32;
    // the fused post pass's FS instance replays the best path's 128 leaves in the frame's region
    // (208 doubles at L = 8; at L = 4 the stride grows 120 -> 152, still = 24 mod 32)
    static constexpr int FSTRIDE_FS = FSTRIDE >= 128 ? FSTRIDE : FSTRIDE + 32;
    // the exact instance (EX) adds a frame's routing slots (16 ints: a survivor's code by list position)
    static constexpr int FSTRIDE_EX = FSTRIDE + 8;
};

// monotone map of an fp64 to uint64 (total order of non-NaN values, -0 == +0), as dlscl.hip
__device__ __forceinline__ uint64_t flip_order_key(double q) {
    if (q == 0.0) q = 0.0;
    const uint64_t u = pscl_asu64(q);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}

// L = 4: keep the lane's 32 channel LLRs in registers across the frame (1) or re-read them at each
// depth-1..3 recompute (0).  Measured (tools/ab_bench.sh, config 2, two rounds): 1.649 / 1.655 ms
// against 1.672 / 1.668
#ifndef PSCL_LANE_CREG4
#define PSCL_LANE_CREG4 1
#endif

// timing-only ablations of the plain kernel (tools/build_variant.py; 0 in the product): 1 every
// full-list information phase ranked (outputs still exact), 2 never ranked (invalid outputs), 4 no
// depth-1..3 recompute (invalid), 8 no epilogue table lookups (invalid)
#ifndef PSCL_LANE_ABL
#define PSCL_LANE_ABL 0
#endif

#ifndef PSCL_LANE_WAVES_PER_EU
#define PSCL_LANE_WAVES_PER_EU 2
#endif

// FS: the DL-SCL retry decodes (dlscl.hip, capi.cpp dl_retry_chunk) -- a round's entries read
// bucket by bucket (P.elist), LLR rows by indirection (P.fidx), forced information bits (P.force:
// the reference bits below the flip index, the flipped bit at it, scl.py:146-161) and the warm
// start at the first 16-phase segment of the wavefront's bucket (P.warm_metric / P.warm_u, the
// forced prefix's exact metric and bits written by the post pass).  The list of a frame then
// grows from one path at its own phases: each frame carries its live-path count (lcnt = log2),
// and an information phase is, per frame, forced (the single path takes the forced child, no
// ordering decision), growing (every child survives) or full (the keep / one-swap / ranked
// tiers, their certificates restricted to the full frames).  Frames it cannot certify go to
// the deferred bucket lists (P.amb_elist, flags PSCL_DL_DEFERRED) for the exact FS kernel.
// channel_kernel's phase A for frame counter fr (scl_kernels.hip): the payload draw (raw, for the
// uncoded baseline), the message (payload + CRC remainder, crc.py:19-37) and the codeword
// (polar.py:17-29,106-119) by the handle's byte tables
__device__ __forceinline__ void tx_frame_words(const pscl_decode_params& P, uint64_t fr, uint64_t (&m)[2],
                                               uint64_t (&raw)[2], uint64_t (&x)[2]) {
    const u32x4 rb = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), 0xffffffffu, 0u}, P.tx_k0, P.tx_k1);
    raw[0] = ((uint64_t)rb.y << 32) | rb.x;
    raw[1] = ((uint64_t)rb.w << 32) | rb.z;
    const int kp = P.tx_kp, nbp = (kp + 7) >> 3, nb = (P.K + 7) >> 3;
    m[0] = kp >= 64 ? raw[0] : (raw[0] & ((1ULL << kp) - 1));
    m[1] = kp > 64 ? (raw[1] & ((kp >= 128) ? ~0ULL : ((1ULL << (kp - 64)) - 1))) : 0;
    uint32_t rem = 0;
    for (int k = 0; k < nbp; ++k) rem ^= P.tx_crctab[k * 256 + (uint32_t)((m[k >> 3] >> (8 * (k & 7))) & 255u)];
    if (P.tx_crc_deg) {
        const uint64_t rw = (uint64_t)rem;
        if (kp < 64) {
            m[0] |= rw << kp;
            if (kp + P.tx_crc_deg > 64) m[1] |= rw >> (64 - kp);
        } else {
            m[1] |= rw << (kp - 64);
        }
    }
    x[0] = x[1] = 0;
    for (int k = 0; k < nb; ++k) {
        const uint32_t v = (uint32_t)((m[k >> 3] >> (8 * (k & 7))) & 255u);
        x[0] ^= P.tx_xtab[(k * 256 + v) * 2];
        x[1] ^= P.tx_xtab[(k * 256 + v) * 2 + 1];
    }
}

// occupancy hint of the L = 8 forced-bit (FS) retry instance: 3 waves per SIMD (168 VGPRs), the plain
// kernel's occupancy; left to the default (2) it took 173
#ifndef PSCL_FS_WAVES
#define PSCL_FS_WAVES 3
#endif
// occupancy hint of the fused TX instance at L = 8: 3 waves per SIMD (168 VGPRs), the plain kernel's
// occupancy (its LDS allows no more); its draws would otherwise take it to ~177 VGPRs and 2 waves
#ifndef PSCL_TX_WAVES
#define PSCL_TX_WAVES 3
#endif
// TXF: the fused TX instance (pscl_simulate_device, PSCL_TUNE_TX_FUSED; P.tx and the tx_* fields of
// pscl_decode_params): each frame's channel row is drawn here from channel_kernel's Philox stream
// -- the same draws, the same fp64 expression, so the decode sees bit for bit the row
// channel_kernel would have written -- instead of being loaded.  The 8 (L = 8) or 4 (L = 4) lanes of
// a frame hold exactly the positions of 8 or 16 whole Box-Muller pairs (pair c gives positions c and
// c + 64; lane p needs p + G k + 16 m), so the frame draws its 64 pairs once, as channel_kernel does;
// every lane of the frame forms the payload, CRC and codeword itself (channel_kernel's phase A,
// byte tables).  Epilogue: the message words of every frame (the reference of the counts and of
// the DL-SCL counter pass), the rows of the frames whose best candidate fails the CRC or that are
// deferred (the retry and exact decodes read them; regenerated, ~1 % of frames at 5 dB), and the
// uncoded BPSK baseline of the same payloads (channel_kernel's draws 0x40000000 + c).
// FP: the FS instance with the fused post pass (P.fpost; its own instantiation -- compiled into the
// plain FS instance behind a runtime flag, the post's registers raised that kernel's peak too,
// L = 8 173 -> 226 VGPRs, L = 4 240 -> 256 + 26 spilled)
// EX: the EXACT lane-per-path decode (pscl_launch_lane_exact): the deferred frames'
// re-decode (plain, rows by P.fidx, outputs at their rows) and the exact forced-bit retry decodes (FS:
// the side chain, unscreened chains).  Natural-log LLR tree, glibc-exact metric tails
// (pscl_softplus_tail_bf), children metrics as scl128_kernel forms them, and the list kept in LIST
// ORDER in the frame's lanes (lane p = list position p): the stable sort's (metric, 2 position + bit)
// order decides every survivor set and position exactly (scl.py:163-174) -- in place when every
// worse child lies above the largest better child and the better children are in order (the keep
// tier), else by ranking the 2L children (each lane counts the keys below its two, DPP-free
// shuffles over the frame's lanes) and routing the survivors through LDS slots; frozen phases
// re-sort only when a metric fell below its predecessor's.  No certificates, no deferral.
template <int LMAX, int CODE, bool FS = false, bool TXF = false, bool FP = false, bool EX = false>
__global__ void __launch_bounds__(64, TXF ? (LMAX == 8 ? PSCL_TX_WAVES : 2)
                                           : (FS && !FP && !EX && LMAX == 8) ? PSCL_FS_WAVES : PSCL_LANE_WAVES_PER_EU)
scl_lane_kernel(const pscl_decode_params P) {
    static_assert(LMAX == 4 || LMAX == 8, "the lane-per-path decoder is built for L = 4 and 8");
    static_assert(!TXF || (!FS && CODE == 1), "fused TX: plain decodes of the (128,64) code");
    static_assert(!FP || (FS && CODE == 1), "fused post pass: the FS instance of the (128,64) code");
    static_assert(!EX || (!TXF && !FP), "the exact instance: plain re-decodes and forced-bit retry decodes");
    using Ly = LaneLayout<LMAX>;
    constexpr int G = Ly::G, F = Ly::F, LOG_G = Ly::LOG_G;
    constexpr int EPL = 16 / G;                 // depth-3 elements per lane at a recompute
    constexpr uint32_t GM = (1u << G) - 1u;     // a frame's bits in a lane mask
    constexpr int K = kSpecK[CODE], PW = (K + 63) / 64;
    constexpr uint64_t info0 = kSpecInfo[CODE][0], info1 = kSpecInfo[CODE][1];
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* const A = reinterpret_cast<double*>(smem);
    const int lane = threadIdx.x & 63;
    // frame fl of the wavefront and path index p of this lane; lane_lo / lane_hi: the frame's lanes
    // of p = 0 and p = 4 (PSCL_LANE_REMAP at L = 8), or its first lane
    constexpr bool REMAP = PSCL_LANE_REMAP && G == 8 && !EX;
    const int rq = (lane >> 2) & 3, inner = (rq == 1 || rq == 2) ? 1 : 0;
    const int fl = REMAP ? 2 * (lane >> 4) + inner : lane >> LOG_G;
    const int p = REMAP ? (lane & 3) + 4 * (rq & 1) : lane & (G - 1);
    const int lane_lo = REMAP ? (lane & ~15) + (inner ? 8 : 0) : lane & ~(G - 1);
    const int lane_hi = REMAP ? (lane & ~15) + (inner ? 4 : 12) : lane_lo + 4;
    // the lane of path index q of this frame
    auto lane_of = [&](uint32_t q) -> int { return REMAP ? (q < 4u ? lane_lo + (int)q : lane_hi + (int)q - 4) : lane_lo + (int)q; };
    double* const Af = A + fl * (FP ? Ly::FSTRIDE_FS : EX ? Ly::FSTRIDE_EX : Ly::FSTRIDE);
    int* const sl = reinterpret_cast<int*>(Af + Ly::FSTRIDE);  // EX: the frame's routing slots
    const uint8_t* const GT = reinterpret_cast<const uint8_t*>(P.epi_table);   // [16][256] u-byte -> info bits
    const uint32_t* const ST = reinterpret_cast<const uint32_t*>(GT + 16 * 256);  // [K/4][16] nibble -> syndrome
    auto hiw = [](double m) { return (uint32_t)(pscl_asu64(m) >> 32); };
    // the margin-raised key hi(fma(m, 1 + 2^-40, MARGIN)) as one VOP3 fma with the factor in an SGPR
    // (left to itself the compiler emits a copy of the margin register plus v_fmac_f64)
    constexpr bool BITS = !FS && !EX && PSCL_LANE_BITS;
    constexpr double MARGIN = BITS ? PSCL_TAIL2_MARGIN : PSCL_TAIL_ABS_MARGIN;
    auto hiw_up = [&](double m) {
        double r;
        asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(m), "s"(1.0 + 0x1p-40), "v"(MARGIN));
        return hiw(r);
    };
    // this frame's G bits of a wave ballot (one 64-bit shift by the frame's first lane)
    auto frame_bits = [&](uint64_t m) -> uint32_t {
        if constexpr (REMAP) return ((uint32_t)(m >> lane_lo) & 15u) | (((uint32_t)(m >> lane_hi) & 15u) << 4);
        return (uint32_t)(m >> lane_lo) & GM;
    };

    int cfe = 0, cbe = 0, cpe = 0, cpb = 0;  // this lane's error counts (flushed at the end)
    int tufe = 0, tube = 0;                  // TXF: the uncoded baseline's errors
    int pdecodes = 0;                        // FS with the fused post pass: attempts recorded
    // frames of the launch: P.B, or (FS) the total of the round's bucket lists
    int bpre[PSCL_DL_NSEG + 1];
    int64_t Bn = P.B;
    if constexpr (FS) {
        const int64_t tot = pscl_bucket_prefix(P.bcount, P.bcap, bpre);
        Bn = tot < P.B ? tot : P.B;
    } else if constexpr (EX) {  // (the re-decode: the first *d_count listed frames)
        if (P.d_count) Bn = *P.d_count < P.B ? (int64_t)*P.d_count : P.B;
    }
    for (int64_t f0 = (int64_t)blockIdx.x * F; f0 < Bn; f0 += (int64_t)gridDim.x * F) {
        const int64_t fi = f0 + fl;
        const bool fvalid = fi < Bn;
        const int64_t fsafe = fvalid ? fi : f0;  // (a tail wave's empty slots decode a copy of frame f0)
        // FS: f = the entry id (force words, warm state, outputs), frow = its LLR row; seg0 = the
        // warm-start segment (wave-uniform: the bucket of the wavefront's first entry -- later
        // entries sit in the same or a later bucket, so every frame is still forced there)
        int64_t f = fi, frow = fsafe;
        int seg0 = 0;
        if constexpr (FS) {
            f = pscl_elist_entry(P, fsafe, bpre);
            seg0 = pscl_bucket_of(f0, bpre);
            frow = P.fidx[f];
        } else if constexpr (EX) {
            if (P.fidx) frow = P.fidx[fsafe];
        }
        // CODE = 2 (the NR (128,88) code, config 5): the input rows are rate matched -- E received
        // LLRs, de-rate-matched and de-interleaved per position as the values are loaded
        constexpr bool RM = CODE == 2;
        const double* chan = P.llr + frow * (RM ? (int64_t)P.rm_E : (int64_t)kN);
        auto chan_at = [&](int i) -> double { return RM ? nr_stage(chan, P.rm_src[i], P.rm_E, kN) : chan[i]; };
        // the frame's channel LLRs in registers: the lane's depth-3 elements e_k = p + G k (k < EPL)
        // need c[8 k + m] = chan[e_k + 16 m] -- the same at all 8 depth-1..3 recomputes
        // (CREG = false, an L = 4 build option: the 32 values are re-read from the L2-resident row at
        // each recompute instead, which keeps them out of the registers of the other phases)
        constexpr bool CREG = G == 8 || PSCL_LANE_CREG4 || TXF;
        double c[8 * EPL];
        // fused TX: the frame's payload draw, message and codeword words (channel_kernel phase A)
        uint64_t tm[2] = {0, 0}, traw[2] = {0, 0}, tx[2] = {0, 0};
        const uint64_t tfr = TXF ? (uint64_t)(P.tx_frame0 + fsafe) : 0ULL;
        if constexpr (TXF) tx_frame_words(P, tfr, tm, traw, tx);
        // the channel values of this lane's positions e = p + G k + 16 m, unscaled (the fused TX
        // instance; channel_kernel's row[e]): pair blk = p + G k + 16 j gives m = j and m = j + 4
        auto gen_chan = [&](double* v, uint64_t fr) {
#pragma unroll
            for (int k = 0; k < EPL; ++k)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t blk = (uint32_t)(p + G * k + 16 * j);
                    const u32x4 rn = philox4x32(u32x4{(uint32_t)fr, (uint32_t)(fr >> 32), blk, 0u}, P.tx_k0, P.tx_k1);
                    double z[2];
                    bm_pair(((uint64_t)rn.y << 32) | rn.x, ((uint64_t)rn.w << 32) | rn.z, z[0], z[1]);
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const double sym = ((tx[h] >> blk) & 1ULL) ? -1.0 : 1.0;
                        v[8 * k + j + 4 * h] = (sym + P.tx_sigma * z[h]) * P.tx_scale;
                    }
                    // one pair at a time: interleaved, the 8 (16) Philox chains' temporaries raise the
                    // kernel's register peak above the decode's own
                    __builtin_amdgcn_sched_barrier(0);
                }
        };
        auto load_chan = [&]() {
            if constexpr (TXF) {
                gen_chan(c, tfr);
                if constexpr (BITS)
#pragma unroll
                    for (int m = 0; m < 8 * EPL; ++m) c[m] = c[m] * PSCL_LOG2E_F64;
            } else {
#pragma unroll
                for (int k = 0; k < EPL; ++k)
#pragma unroll
                    for (int m = 0; m < 8; ++m) c[8 * k + m] = BITS ? chan_at(p + G * k + 16 * m) * PSCL_LOG2E_F64
                                                                    : chan_at(p + G * k + 16 * m);
            }
        };
        load_chan();
        if constexpr (TXF) {
            // the uncoded BPSK baseline of the same payload (channel_kernel phase A: noise pairs
            // 0x40000000 + cb), counted here while the decode's registers are still free
            if (P.tx_upart) {
                uint32_t berr = 0;
                for (int cb = p; 2 * cb < P.tx_kp; cb += G) {
                    const u32x4 rn = philox4x32(u32x4{(uint32_t)tfr, (uint32_t)(tfr >> 32), 0x40000000u + (uint32_t)cb, 0u},
                                                P.tx_k0, P.tx_k1);
                    double z[2];
                    bm_pair(((uint64_t)rn.y << 32) | rn.x, ((uint64_t)rn.w << 32) | rn.z, z[0], z[1]);
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int q = 2 * cb + h;
                        if (q < P.tx_kp) {
                            const uint32_t bit = (uint32_t)((traw[q >> 6] >> (q & 63)) & 1ULL);
                            const double y = (bit ? -1.0 : 1.0) + P.tx_unc_sigma * z[h];
                            berr += ((y < 0.0) ? 1u : 0u) != bit ? 1u : 0u;
                        }
                    }
                }
                berr = frame_sum<G>(berr);
                if (fvalid && p == 0) {
                    tufe += berr ? 1 : 0;
                    tube += (int)berr;
                }
            }
        }
        // frames whose channel magnitudes could overflow the fp64 metric sums or carry a NaN go to
        // the exact re-decode (the lane's values summed; NaN propagates through the sum); in bits,
        // a tighter bound keeps the scaled tree's error below PSCL_TAIL2_TREE (glibc_softplus.h)
        double cs = fabs(c[0]);
#pragma unroll
        for (int m = 1; m < 8 * EPL; ++m) cs = cs + fabs(c[m]);
        uint64_t amb = EX ? 0ULL : wmask(!(cs < (BITS ? PSCL_TAIL2_CHAN_SUM : 0x1p25)));
        const uint64_t vmask = wmask(fvalid);

        double metric = 0.0;
        uint64_t u0 = 0, u1 = 0;  // decided bits
        uint32_t tab = 0;          // LDS slot of depths 3..6 (4 bits each)
        uint32_t lastbit = 0;      // the bit decided at the previous phase
        double r5[4] = {0.0, 0.0, 0.0, 0.0}, r6[2] = {0.0, 0.0};  // PSCL_LANE_REG56: depths 5 and 6 of this lane's path
        uint64_t fm0 = 0, fm1 = 0, fv0 = 0, fv1 = 0;  // FS: force mask and values (information bits)
        int lcnt = 0;                                 // FS: log2 of the frame's live paths
        if constexpr (FS) {
            const uint64_t* fr = P.force + f * 2 * PW;
            fm0 = fr[0];
            fv0 = fr[PW];
            if (PW > 1) {
                fm1 = fr[1];
                fv1 = fr[PW + 1];
            }
            // warm start at phase 16 seg0: one path, its exact metric and bits below that phase
            if (seg0 > 0) {
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

        auto phase = [&](auto PC) {
            constexpr int phi = decltype(PC)::value;
            constexpr int t = phi & 15;
            constexpr int start = t ? kn - __builtin_ctz((unsigned)t) : ((phi >> 4) ? 3 - __builtin_ctz((unsigned)(phi >> 4)) : 1);
            constexpr bool is_info = ((phi < 64 ? info0 : info1) >> (phi & 63)) & 1;
            constexpr int jb = phi < 64 ? __builtin_popcountll(info0 & ((1ULL << (phi & 63)) - 1))
                                        : __builtin_popcountll(info0) + __builtin_popcountll(info1 & ((1ULL << (phi & 63)) - 1));
            constexpr int cnt = jb >= LOG_G ? LMAX : (1 << jb);  // live paths (min(2^j, L))
#ifdef PSCL_PHASE_MARKERS  // asm listing analysis only (tools/isa_phase_stats.py)
            asm volatile("; PHASE %0" ::"n"(t));
#endif

            // ---- depths 1-3 recomputed from the channel (phi % 16 == 0)
            if constexpr (start <= 3 && !(PSCL_LANE_ABL & 4)) {
                constexpr bool r1 = phi >= 64, r2 = (phi >> 5) & 1, r3 = (phi >> 4) & 1;
                if constexpr (!CREG && phi > 0) load_chan();
                uint4* const xs = reinterpret_cast<uint4*>(Af + Ly::OFFX);
                if constexpr (r1 || r2 || r3) {
                    uint64_t X1 = 0;
                    uint32_t X2 = 0, X3 = 0;
                    if (r1) X1 = polar_transform64(u0);
                    if (r2) {
                        constexpr int lo = phi - (phi & 31) - 32;
                        X2 = polar_transform32((uint32_t)((lo >= 64 ? u1 : u0) >> (lo & 63)));
                    }
                    if (r3) {
                        constexpr int lo = phi - 16;
                        X3 = polar_transform16((uint32_t)((lo >= 64 ? u1 : u0) >> (lo & 63)) & 0xffffu);
                    }
                    // (X2 with X3 as the 64-bit word [X2, X2 >> 16 | X3 << 16]: bit e of X2 and bit e + 16
                    // land on bit 31 of the two halves by one 64-bit shift, bit e of X3 is bit e + 16
                    // of the high half)
                    xs[p] = make_uint4((uint32_t)X1, (uint32_t)(X1 >> 32), X2, (X2 >> 16) | (X3 << 16));
                    wave_lds_fence();
                }
                // the depth-1 f node is the same for every path before phase 64, and depth 2 too
                // at phases 0 and 16
                constexpr bool shared2 = !r1 && !r2;
                double d1l[EPL][4], d2s[EPL][2];
#pragma unroll
                for (int h = 0; h < EPL; ++h) {
#pragma unroll
                    for (int m = 0; m < 4; ++m) d1l[h][m] = r1 ? 0.0 : f_minsum(c[8 * h + m], c[8 * h + m + 4]);
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) d2s[h][s2] = shared2 ? f_minsum(d1l[h][s2], d1l[h][s2 + 2]) : 0.0;
                }
                constexpr int npaths = FS ? LMAX : cnt;  // (FS: the frames' list sizes differ)
#pragma unroll
                for (int q0 = 0; q0 < npaths; ++q0) {
                    // lane p takes path (q0 + p) mod L: the 8 lanes' stores hit 8 distinct bank groups
                    const int q = npaths == LMAX ? ((q0 + p) & (LMAX - 1)) : q0;
                    uint64_t x1 = 0, x23 = 0;
                    if constexpr (r1 || r2 || r3) {
                        const uint4 xv = xs[q];
                        x1 = ((uint64_t)xv.y << 32) | xv.x;
                        x23 = ((uint64_t)xv.w << 32) | xv.z;
                    }
                    double d3[EPL];
#pragma unroll
                    for (int h = 0; h < EPL; ++h) {
                        const uint32_t e = (uint32_t)(p + G * h);
                        // the g nodes' bits moved to bit 31 of a 32-bit half by 64-bit shifts, each
                        // serving two nodes: bits e + 16 s and e + 16 s + 32 of X1 (depth 1), bits e and
                        // e + 16 of X2 (depth 2)
                        const uint64_t s1[2] = {r1 ? x1 << (31u - e) : 0ULL, r1 ? x1 << (15u - e) : 0ULL};
                        const uint64_t s2w = r2 ? x23 << (31u - e) : 0ULL;
                        double d1[4];
#pragma unroll
                        for (int m = 0; m < 4; ++m)
                            d1[m] = r1 ? g_node_bit31(c[8 * h + m], c[8 * h + m + 4], (uint32_t)(s1[m & 1] >> (32 * (m >> 1))))
                                       : d1l[h][m];
                        double d2[2];
#pragma unroll
                        for (int s2 = 0; s2 < 2; ++s2)
                            d2[s2] = shared2 ? d2s[h][s2]
                                             : (r2 ? g_node_bit31(d1[s2], d1[s2 + 2], (uint32_t)(s2w >> (32 * s2))) : f_minsum(d1[s2], d1[s2 + 2]));
                        d3[h] = r3 ? g_node_wbit(d2[0], d2[1], (uint32_t)(x23 >> 32), e + 16) : f_minsum(d2[0], d2[1]);
                    }
                    // elements e_k and e_k + 8 = e_{k + EPL/2} of slot q: one pair ([8][L][2] layout)
#pragma unroll
                    for (int h = 0; h < EPL / 2; ++h)
                        *reinterpret_cast<double2*>(Af + Ly::OFF3 + ((p + G * h) * LMAX + q) * 2) = make_double2(d3[h], d3[h + EPL / 2]);
                }
                wave_lds_fence();
            }
            // ---- depths 4..6: this lane's own path; the first rewritten depth reads the parent slot
            if constexpr (start <= 6) {
                uint32_t xsb = 0;  // partial sums of the first rewritten node's left sibling (g node)
                if constexpr (phi && start >= 4) {
                    constexpr int w = 1 << (kn - start), lo = phi - w;
                    xsb = polar_transform8((uint32_t)((lo >= 64 ? u1 : u0) >> (lo & 63)) & ((1u << w) - 1u));
                }
                static_for<3>([&](auto DI) {
                    constexpr int D = 4 + decltype(DI)::value;
                    if constexpr (D >= start) {
                        constexpr int W = 1 << (kn - D), HW = W / 2;
                        constexpr int OFF_IN = D == 4 ? Ly::OFF3 : (D == 5 ? Ly::OFF4 : Ly::OFF5);
                        constexpr int OFF_OUT = D == 4 ? Ly::OFF4 : (D == 5 ? Ly::OFF5 : Ly::OFF6);
                        constexpr bool first = D == start || (D == 4 && start < 4);
                        constexpr bool is_g = D == start && phi != 0;
                        if constexpr (PSCL_LANE_REG56 && D == 6) {
                            // from this path's depth-5 registers (computed this phase, or carried
                            // along with the path since)
#pragma unroll
                            for (int k = 0; k < 2; ++k)
                                r6[k] = is_g ? g_node(r5[k], r5[k + 2], (xsb >> k) & 1u) : f_minsum(r5[k], r5[k + 2]);
                        } else {
                            const int sin = first ? slot_at(tab, D - 1) : p;  // (depth 3 at a recompute: own slot p)
                            const int sin_eff = (D == 4 && start <= 3) ? p : sin;
                            const double* in = Af + OFF_IN + sin_eff * 2;
                            double o[W];
#pragma unroll
                            for (int k = 0; k < W; ++k) {
                                const double2 ab = *reinterpret_cast<const double2*>(in + k * LMAX * 2);
                                o[k] = is_g ? g_node(ab.x, ab.y, (xsb >> k) & 1u) : f_minsum(ab.x, ab.y);
                            }
                            if constexpr (PSCL_LANE_REG56 && D == 5) {
#pragma unroll
                                for (int k = 0; k < 4; ++k) r5[k] = o[k];
                            } else {
                                double* out = Af + OFF_OUT + p * 2;
                                if constexpr (HW >= 1) {
#pragma unroll
                                    for (int k = 0; k < (HW ? HW : 1); ++k)
                                        *reinterpret_cast<double2*>(out + k * LMAX * 2) = make_double2(o[k], o[k + HW]);
                                }
                                wave_lds_fence();
                            }
                        }
                    }
                });
                // this path's own slot at every depth rewritten this phase
                constexpr int s0 = start < 3 ? 3 : start;
                constexpr uint32_t mask = (0xffffu << (4 * (s0 - 3))) & 0xffffu;
                tab = (tab & ~mask) | ((uint32_t)p * 0x1111u & mask);
            }
            // ---- leaf LLR and metric tail (scl.py:80-82, 102-105)
            const double2 lab = PSCL_LANE_REG56 ? make_double2(r6[0], r6[1])
                                                : *reinterpret_cast<const double2*>(Af + Ly::OFF6 + (start <= 6 ? p : slot_at(tab, 6)) * 2);
            // a lane taking another path's child also takes that path's depth-6 node (needed by the
            // next, odd, leaf: even phases) and its depth-5 node (needed by the depth-6 g node two
            // phases on: phases 0 and 1 mod 4)
            constexpr bool C6 = PSCL_LANE_REG56 && (t % 2 == 0), C5 = PSCL_LANE_REG56 && (t % 4 <= 1);
            auto carry = [&](int src, double (&q5)[4], double (&q6)[2]) {
                if constexpr (C5)
#pragma unroll
                    for (int k = 0; k < 4; ++k) q5[k] = shfl_f64(r5[k], src);
                if constexpr (C6)
#pragma unroll
                    for (int k = 0; k < 2; ++k) q6[k] = shfl_f64(r6[k], src);
            };
            auto take = [&](const double (&q5)[4], const double (&q6)[2]) {
                if constexpr (C5)
#pragma unroll
                    for (int k = 0; k < 4; ++k) r5[k] = q5[k];
                if constexpr (C6)
#pragma unroll
                    for (int k = 0; k < 2; ++k) r6[k] = q6[k];
            };
            const double lam = (phi & 1) ? g_node(lab.x, lab.y, lastbit) : f_minsum(lab.x, lab.y);
            const double Lt = EX ? pscl_softplus_tail_bf(lam, P.exp_table) : BITS ? pscl_softplus_tail2(lam) : pscl_softplus_tail_abs(lam);
            if constexpr (EX) {
                // ---- exact: lanes 0..ncur-1 of the frame hold its live paths in list order
                const int ncur = FS ? (1 << lcnt) : cnt;
                const bool live = p < ncur;
                const bool zl = lam == 0.0;
                // the whole state of lane src's path (its metric chosen by the caller)
                auto pull_path = [&](int src) {
                    u0 = shfl_u64(u0, src);
                    if constexpr (phi >= 64) u1 = shfl_u64(u1, src);
                    tab = bperm32(tab, src);
                    double q5[4], q6[2];
                    carry(src, q5, q6);
                    take(q5, q6);
                };
                if constexpr (!is_info) {  // bit 0 (scl.py:149-153), then the list re-sorted stably
                    metric = zl ? metric + PSCL_LOGE2 : metric + (relu_neg(lam) + Lt);
                    lastbit = 0;
                    const double pm = shfl_f64(metric, p > 0 ? lane - 1 : lane);
                    if ((wmask(live && pm > metric) & vmask) == 0) return;
                    const double mk = live ? metric : __builtin_inf();
                    uint32_t r = 0;
#pragma unroll
                    for (int sx = 1; sx < G; ++sx) {
                        const double om = shfl_f64(mk, lane ^ sx);
                        r += (om < mk || (om == mk && (p ^ sx) < p)) ? 1u : 0u;
                    }
                    if (live) sl[r] = p;
                    wave_lds_fence();
                    const int src = lane_lo + sl[p & (ncur - 1)];  // (lanes beyond the list: copies)
                    wave_lds_fence();
                    metric = shfl_f64(metric, src);
                    pull_path(src);
                    return;
                }
                // children metrics as scl128_kernel forms them (scl.py:102-105): along the LLR sign
                // metric + L, against it metric + (|lam| + L); an exactly zero LLR both metric + ln 2
                const bool neg = lam < 0.0;
                const double mgd = metric + Lt, mbd = metric + (fabs(lam) + Lt);
                double m0 = neg ? mbd : mgd, m1 = neg ? mgd : mbd;
                if (zl) {
                    m0 = metric + PSCL_LOGE2;
                    m1 = m0;
                }
                bool forced = false;
                uint32_t fbit = 0;
                if constexpr (FS) {
                    const uint64_t fmw = jb < 64 ? fm0 : fm1, fvw = jb < 64 ? fv0 : fv1;
                    forced = ((fmw >> (jb & 63)) & 1ULL) != 0;
                    fbit = (uint32_t)((fvw >> (jb & 63)) & 1ULL);
                }
                // frames decided without ranking: a forced single path takes the forced child; a
                // full list keeps its better children in place when they stay in order and every
                // worse child lies strictly above the largest of them (the stable sort's outcome)
                const double top = shfl_f64(mgd, lane_lo + LMAX - 1), pg = shfl_f64(mgd, p > 0 ? lane - 1 : lane);
                const bool badk = zl || (p > 0 && pg > mgd) || !(mbd > top);
                const bool fast = forced ? ncur == 1 : (ncur == LMAX && frame_bits(wmask(badk)) == 0);
                uint32_t b = forced ? fbit : sign_bit(lam);
                if ((wmask(!fast) & vmask) != 0) {
                    // rank the frame's valid children on (metric, 2 position + bit); the first ncnt
                    // survive at list positions = their ranks (scl.py:163-174)
                    const bool v0 = live && (!forced || fbit == 0u), v1 = live && (!forced || fbit == 1u);
                    const int ncnt = forced ? ncur : (2 * ncur < LMAX ? 2 * ncur : LMAX);
                    const double k0 = v0 ? m0 : __builtin_inf(), k1 = v1 ? m1 : __builtin_inf();
                    uint32_t r0 = k1 < k0 ? 1u : 0u, r1 = k0 <= k1 ? 1u : 0u;
#pragma unroll
                    for (int sx = 1; sx < G; ++sx) {
                        const double o0 = shfl_f64(k0, lane ^ sx), o1 = shfl_f64(k1, lane ^ sx);
                        const bool lt = (p ^ sx) < p;
                        r0 += ((o0 < k0 || (o0 == k0 && lt)) ? 1u : 0u) + ((o1 < k0 || (o1 == k0 && lt)) ? 1u : 0u);
                        r1 += ((o0 < k1 || (o0 == k1 && lt)) ? 1u : 0u) + ((o1 < k1 || (o1 == k1 && lt)) ? 1u : 0u);
                    }
                    if (!fast) {
                        if (v0 && r0 < (uint32_t)ncnt) sl[r0] = 2 * p;
                        if (v1 && r1 < (uint32_t)ncnt) sl[r1] = 2 * p + 1;
                    }
                    wave_lds_fence();
                    const int code = fast ? 2 * p + (int)b : sl[p & (ncnt - 1)];  // (beyond the list: copies)
                    wave_lds_fence();
                    const int src = lane_lo + (code >> 1);
                    b = (uint32_t)code & 1u;
                    const double p0 = shfl_f64(m0, src), p1 = shfl_f64(m1, src);
                    metric = b ? p1 : p0;
                    pull_path(src);
                    if constexpr (FS) lcnt += (!fast && !forced && ncur < LMAX) ? 1 : 0;
                } else {
                    metric = b ? m1 : m0;
                }
                if (phi < 64) u0 |= (uint64_t)b << phi; else u1 |= (uint64_t)b << (phi - 64);
                lastbit = b;
                return;
            }
            if constexpr (!is_info) {  // frozen: bit 0 (scl.py:149-153)
                metric = metric + (relu_neg(lam) + Lt);
                lastbit = 0;
                return;
            }
            // information phase: better child (along the LLR sign) mg, worse child mb
            const double mg = metric + Lt, mb = mg + fabs(lam);
            const uint32_t gbit = sign_bit(lam);
            if constexpr (FS) {
                // per frame: forced, growing or full (frame-uniform); the own child first, then the
                // lanes that take another path's child pull it in one exchange
                const uint64_t fmw = jb < 64 ? fm0 : fm1, fvw = jb < 64 ? fv0 : fv1;
                const bool forced = ((fmw >> (jb & 63)) & 1ULL) != 0;
                const uint32_t fbit = (uint32_t)((fvw >> (jb & 63)) & 1ULL);
                const bool full = !forced && lcnt == LOG_G, grow = !forced && lcnt < LOG_G;
                const int cntf = 1 << lcnt;
                const double m1 = gbit ? mg : mb;  // the bit-1 child
                double nm = forced ? (fbit == gbit ? mg : mb) : (grow ? (gbit ? mb : mg) : mg);
                uint32_t b = forced ? fbit : (grow ? 0u : gbit);
                // growing: bit-1 children to lanes cnt..2cnt-1
                bool pull = grow && (p & cntf) != 0;
                int src = grow ? lane_of((uint32_t)(p & (cntf - 1))) : lane;
                const uint64_t fullm = wmask(full) & vmask;
                const uint32_t kgu = hiw_up(mg), kb = hiw(mb);
                const uint32_t mx = frame_max<G>(kgu);
                const bool bad = kb <= mx;
                const uint64_t badm = wmask(bad);
                if ((badm & fullm) != 0) {  // some full frame has a worse child within the margin
                    const uint32_t bad8 = frame_bits(badm);
                    if ((wmask(__builtin_popcount(bad8) > 1) & fullm) == 0) {
                        // one swap per full frame at most (see the plain form below)
                        const uint32_t kg = hiw(mg);
                        const uint32_t gmaxh = frame_max<G>(kg);
                        const bool ismax = kg == gmaxh;
                        const uint32_t nmax = frame_sum<G>(ismax ? 1u : 0u);
                        const uint32_t g2u = frame_max<G>(ismax ? 0u : kgu);
                        const uint32_t wu = frame_max<G>(bad ? hiw_up(mb) : 0u);
                        const bool swap = bad8 != 0;
                        amb |= wmask(full && swap && !(nmax == 1u && g2u < gmaxh && wu < gmaxh)) & vmask;
                        if (full && swap && ismax) {
                            pull = true;
                            src = lane_of(__builtin_ctz(bad8 | (1u << G)) & (G - 1));
                        }
                    } else {
                        // rank the 2L children of each frame (see the plain form below)
                        const uint32_t kg = hiw(mg);
                        bool keep_g, win_b;
                        select_survivors<G, LMAX>(kg, kb, keep_g, win_b);
                        const uint32_t kbu = hiw_up(mb);
                        const uint32_t su = keep_g ? (win_b ? kbu : kgu) : (win_b ? kbu : 0u);
                        const uint32_t nmk = keep_g ? (win_b ? 0xffffffffu : kb) : kg;
                        const uint32_t nsurv = frame_sum<G>((keep_g ? 1u : 0u) + (win_b ? 1u : 0u));
                        const uint32_t smax = frame_max<G>(su), nmin = frame_min<G>(nmk);
                        amb |= wmask(full && !(nsurv == (uint32_t)LMAX && nmin > smax)) & vmask;
                        const uint32_t f8 = frame_bits(wmask(!keep_g)), w8 = frame_bits(wmask(win_b));
                        const uint32_t jj = __builtin_popcount(f8 & ((1u << p) - 1u));
                        const int rsrc = lane_of(nth_set_bit8(w8, jj));
                        if (full && !keep_g) {
                            pull = true;
                            src = rsrc;
                        }
                    }
                }
                if (wmask(pull) != 0) {
                    // the child a puller takes: a full frame's worse child, a growing frame's bit-1
                    // child; its bit rides on the table word
                    const uint64_t pubm = pscl_asu64(full ? mb : m1);
                    const uint32_t tw = tab | ((full ? (gbit ^ 1u) : 1u) << 31);
                    const uint64_t pm = shfl_u64(pubm, src);
                    const uint64_t pu0 = shfl_u64(u0, src);
                    const uint64_t pu1 = phi >= 64 ? shfl_u64(u1, src) : 0ULL;
                    const uint32_t ptw = bperm32(tw, src);
                    double q5[4], q6[2];
                    carry(src, q5, q6);
                    if (pull) {
                        nm = pscl_asf64(pm);
                        u0 = pu0;
                        u1 = pu1;
                        tab = ptw & 0x7fffffffu;
                        b = ptw >> 31;
                        take(q5, q6);
                    }
                }
                metric = nm;
                if (phi < 64) u0 |= (uint64_t)b << phi; else u1 |= (uint64_t)b << (phi - 64);
                lastbit = b;
                lcnt += grow ? 1 : 0;
                return;
            }
            if constexpr (cnt < LMAX) {
                // growing list: every child survives; bit-1 children to lanes cnt..2cnt-1
                const double m0 = gbit ? mb : mg, m1 = gbit ? mg : mb;
                const int src = lane_of((uint32_t)(p & (cnt - 1)));
                const uint32_t b = (p & cnt) ? 1u : 0u;
                const uint64_t pm1 = shfl_u64(pscl_asu64(m1), src);
                metric = b ? pscl_asf64(pm1) : m0;
                u0 = shfl_u64(u0, src);
                if (phi >= 64) u1 = shfl_u64(u1, src);
                tab = bperm32(tab, src);
                double q5[4], q6[2];
                carry(src, q5, q6);
                take(q5, q6);
                if (phi < 64) u0 |= (uint64_t)b << phi; else u1 |= (uint64_t)b << (phi - 64);
                lastbit = b;
                return;
            }
            // full list: keep the better children when every worse child clears the largest
            // better child by the margin (the stable sort's outcome; ties never reach the sort)
            const uint32_t kgu = hiw_up(mg), kb = hiw(mb);
            const uint32_t mx = frame_max<G>(kgu);
            const bool bad = kb <= mx;  // this worse child is not clear of every better child
            const uint64_t badm = wmask(bad);
#ifdef PSCL_STATS  // diagnostic build (tools/fastpath_stats.py): full-list info phases per wave by
                   // tier: counters[12] kept in place, [13] one swap, [14] full ranking
            const bool one = (wmask(__builtin_popcount(frame_bits(badm)) > 1) & vmask) == 0;
            if (lane == 0 && P.counters) {
                atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + ((badm & vmask) == 0 ? 12 : (one ? 13 : 14)), 1ULL);
            }
#endif
            // the better child stays in place unless a tier below makes this lane pull another
            // path's worse child (the keep tier: no lane pulls)
            metric = mg;
            uint32_t b = gbit;
            if (!(PSCL_LANE_ABL & 2) && ((badm & vmask) != 0 || (PSCL_LANE_ABL & 1))) {
                const uint32_t bad8 = frame_bits(badm);
                bool pull;
                int src;
#if PSCL_LANE_SWAP
                // one-swap tier (every frame of the wave has at most one worse child w that is not
                // clear): the survivors are the better children but the largest, gmax, plus w --
                // certain when w and the second-largest better child are both below gmax by the
                // margin (every other worse child already clears every better child, hence w too);
                // else the frame is deferred (its boundary is within the margin, which no ranking
                // could certify either)
                if (!(PSCL_LANE_ABL & 1) && (wmask(__builtin_popcount(bad8) > 1) & vmask) == 0) {
                    const uint32_t kg = hiw(mg);
                    const uint32_t gmaxh = frame_max<G>(kg);
                    const bool ismax = kg == gmaxh;
                    const uint32_t nmax = frame_sum<G>(ismax ? 1u : 0u);
                    const uint32_t g2u = frame_max<G>(ismax ? 0u : kgu);
                    const uint32_t wu = frame_max<G>(bad ? hiw_up(mb) : 0u);
                    const bool swap = bad8 != 0;
                    amb |= wmask(swap && !(nmax == 1u && g2u < gmaxh && wu < gmaxh)) & vmask;
                    src = lane_of(__builtin_ctz(bad8 | (1u << G)) & (G - 1));  // (frames without a swap: unused)
                    pull = swap && ismax;
                } else
#endif
                {
                    // rank the 2L children of each frame (select_survivors), then certify: exactly L
                    // survivors, and the largest survivor (raised by the margin) below the smallest
                    // non-survivor
                    const uint32_t kg = hiw(mg);
                    bool keep_g, win_b;
                    select_survivors<G, LMAX>(kg, kb, keep_g, win_b);
#if defined(PSCL_STATS) && PSCL_STATS == 2  // diagnostic: ranked-tier frames by surviving worse children
                    {                        // [16 + d] and near-worse count [25 + nb]; waves by max d [34 + d]
                        const uint32_t dw = frame_sum<G>(win_b ? 1u : 0u);
                        const uint32_t nb = __builtin_popcount(bad8);
                        unsigned long long* C = reinterpret_cast<unsigned long long*>(P.counters);
                        if (p == 0 && fvalid && C) {
                            atomicAdd(C + 16 + (dw > 8u ? 8u : dw), 1ULL);
                            atomicAdd(C + 25 + nb, 1ULL);
                        }
                        uint32_t md = 0;
                        for (uint32_t k = 1; k <= 8; ++k)
                            if (wmask(dw >= k) & vmask) md = k;
                        if (lane == 0 && C) atomicAdd(C + 34 + md, 1ULL);
                    }
#endif
                    const uint32_t kbu = hiw_up(mb);
                    const uint32_t su = keep_g ? (win_b ? kbu : kgu) : (win_b ? kbu : 0u);
                    const uint32_t nm = keep_g ? (win_b ? 0xffffffffu : kb) : kg;
                    const uint32_t nsurv = frame_sum<G>((keep_g ? 1u : 0u) + (win_b ? 1u : 0u));
                    const uint32_t smax = frame_max<G>(su), nmin = frame_min<G>(nm);
                    amb |= wmask(!(nsurv == (uint32_t)LMAX && nmin > smax)) & vmask;
                    // freed lanes take the surviving worse children: the j-th freed lane of a frame
                    // pulls the j-th winner (both counted in lane order)
                    const uint32_t f8 = frame_bits(wmask(!keep_g)), w8 = frame_bits(wmask(win_b));
                    const uint32_t j = __builtin_popcount(f8 & ((1u << p) - 1u));
                    src = lane_of(nth_set_bit8(w8, j));
                    pull = !keep_g;
                }
                // the pull: metric, bits and slot table of the source lane's worse child, whose bit
                // rides on the table word
                const uint32_t tw = tab | ((gbit ^ 1u) << 31);
                const uint64_t pmb = shfl_u64(pscl_asu64(mb), src);
                const uint64_t pu0 = shfl_u64(u0, src);
                const uint64_t pu1 = phi >= 64 ? shfl_u64(u1, src) : 0ULL;
                const uint32_t ptw = bperm32(tw, src);
                double q5[4], q6[2];
                carry(src, q5, q6);
                if (pull) {
                    metric = pscl_asf64(pmb);
                    u0 = pu0;
                    u1 = pu1;
                    tab = ptw & 0x7fffffffu;
                    b = ptw >> 31;
                    take(q5, q6);
                }
            }
            if (phi < 64) u0 |= (uint64_t)b << phi; else u1 |= (uint64_t)b << (phi - 64);
            lastbit = b;
        };
        if constexpr (FS) {
            // entered at the warm-start segment: a fall-through switch over the 16-phase segments
            auto seg = [&](auto SB) {
                static_for<16>([&](auto TC) { phase(std::integral_constant<int, decltype(SB)::value * 16 + decltype(TC)::value>{}); });
            };
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
        } else {
            static_for<kN>([&](auto PC) { phase(PC); });
        }

        // ---- the fused post pass of a screened retry round (P.fpost; dl_post_kernel's work, dlscl.hip,
        // for this wavefront's entries, G lanes each: flip.py:97-136).  Per frame: the attempt's
        // best bits, flags and attempt count to the frame (the attempt just decoded is its latest,
        // flip.py:123-136); for a failing frame with flips left, the leaves of its best path replayed
        // top-down in place in the frame's LDS region (bit-identical to the decode's own: f/g of the
        // same values), the next flip -- q = |L0| @ beta, argmin over the untried (q, index),
        // flip.py:104-111, by the packed fp32 sums with dl_post_kernel's certificate, else the exact
        // fp64 sums in index order -- its force words (flip.py:30-34), the warm-start state of its
        // forced prefix (bits, and metrics summed from the screening tail: a screened decode's own,
        // whose per-increment error the certificate already covers), and the append
        // to the next round's bucket list (one atomic per bucket and wavefront).
        auto fused_post = [&](bool x_amb, bool x_live, uint32_t x_keyb, uint32_t x_kbest, uint64_t x_ib0, uint64_t x_ib1,
                              uint64_t x_u0, uint64_t x_u1, int64_t x_frow, int64_t e, bool x_valid) {
            static_assert(!REMAP, "the fused post pass assumes frames of G consecutive lanes");
            const pscl_post_params& Q = P.fp;
            constexpr int NC = K / G;  // flip candidates per lane: j = p + G i
            const uint32_t fl = (x_kbest < (uint32_t)LMAX ? PSCL_FLAG_CRC_PASS : 0u) | (x_kbest & (uint32_t)(LMAX - 1));
            const bool mine = x_valid && !x_amb;  // (deferred frames: the side chain's)
            int nt = 0;
            uint64_t t0 = 0, t1 = 0;
            if (mine) {
                nt = Q.ntried[e];
                t0 = Q.tried[2 * e];
                t1 = Q.tried[2 * e + 1];
            }
            // the best path's lane: its information bits and path bits to every lane of the frame
            const uint32_t bfb = frame_bits(wmask(x_live && x_keyb == x_kbest));
            const int bsrc = lane_lo + (bfb ? __builtin_ctz(bfb) : 0);
            const uint64_t bi0 = shfl_u64(x_ib0, bsrc), bi1 = PW > 1 ? shfl_u64(x_ib1, bsrc) : 0ULL;
            const uint64_t bu0 = shfl_u64(x_u0, bsrc), bu1 = shfl_u64(x_u1, bsrc);
            if (mine && p == 0) {
                Q.best[x_frow * PW] = bi0;
                if (PW > 1) Q.best[x_frow * PW + 1] = bi1;
                Q.flags[x_frow] = (uint8_t)fl;
                if (Q.attempts) Q.attempts[x_frow] = nt + 1;
                ++pdecodes;
            }
            const bool more = mine && !(fl & PSCL_FLAG_CRC_PASS) && nt < Q.rounds;
            if (wmask(more) == 0) return;
            // ---- replay: level d maps the pair (q, q + w) of depth d - 1 to (f, g) in place.  The
            // channel row is read again (L2): kept in the registers c[] until here, it would stay
            // live through the last 16 phases and raise the kernel's register peak by its size
            wave_lds_fence();  // (the decode's last reads of the region)
            {
                const double* crow = P.llr + x_frow * kN;
#pragma unroll
                for (int j = 0; j < kN / G; ++j) Af[p + G * j] = crow[p + G * j];
            }
            wave_lds_fence();
            auto stage = [](uint64_t x, int st) {
                const uint64_t M = st == 1 ? 0x5555555555555555ULL : st == 2 ? 0x3333333333333333ULL
                                 : st == 4 ? 0x0f0f0f0f0f0f0f0fULL : st == 8 ? 0x00ff00ff00ff00ffULL
                                 : st == 16 ? 0x0000ffff0000ffffULL : 0x00000000ffffffffULL;
                return x ^ ((x >> st) & M);
            };
            uint64_t X0 = bu0, X1 = bu1;  // X_lw = u after butterfly stages 1 .. 2^(lw - 1) (dlscl.hip)
#pragma unroll
            for (int mm = 1; mm < kn; ++mm) {
                X0 = stage(X0, 1 << (mm - 1));
                X1 = stage(X1, 1 << (mm - 1));
            }
            // (rolled loops below: unrolled, the compiler issues a whole level's LDS reads before its
            // writes and the kernel's register peak moves here -- 256 VGPRs and spills)
            static_for<kn>([&](auto DC) {
                constexpr int lw2 = kn - 1 - decltype(DC)::value, w2 = 1 << lw2;
                const bool act_l = w2 >= G || (p & w2) == 0;  // (w2 < G: the lane of the pair's first half)
                if (act_l) {
#pragma unroll 2
                    for (int j = 0; j < kN / G; ++j) {
                        const int q = p + G * j;
                        if (w2 >= G && (q & w2)) continue;  // (the pair's second half)
                        const double a = Af[q], b = Af[q + w2];
                        const uint32_t bit = (uint32_t)(((q >> 6) ? X1 : X0) >> (q & 63)) & 1u;
                        Af[q] = f_minsum(a, b);
                        Af[q + w2] = g_node(a, b, bit);
                    }
                }
                wave_lds_fence();
                if constexpr (lw2 > 0) {
                    X0 = stage(X0, w2 >> 1);
                    X1 = stage(X1, w2 >> 1);
                }
            });
            // ---- next flip: q_j = |L0| @ beta (packed fp32, certified) or |L0|
            float qv[NC];  // (fp32 sums, exactly widened; the exact fallback keeps its own fp64 sums)
            double as = 0.0;
            uint64_t bk = ~0ULL;
            int bj = 0x7fffffff;
            auto seen_j = [&](int j) { return (((j < 64 ? t0 : t1) >> (j & 63)) & 1ULL) != 0; };
            auto argmin = [&]() {
                bk = ~0ULL;
                bj = 0x7fffffff;
#pragma unroll
                for (int i = 0; i < NC; ++i) {
                    const int j = p + G * i;
                    const uint64_t key = seen_j(j) ? ~0ULL : flip_order_key((double)qv[i]);
                    if (key < bk) {  // (increasing j: ties keep the lower index)
                        bk = key;
                        bj = j;
                    }
                }
#pragma unroll
                for (int sft = 1; sft < G; sft <<= 1) {
                    const uint64_t ok = shfl_u64(bk, lane ^ sft);
                    const int oj = __shfl(bj, lane ^ sft);
                    if (ok < bk || (ok == bk && oj < bj)) {
                        bk = ok;
                        bj = oj;
                    }
                }
            };
            // exact fallback: index-order sums, each product and sum rounded (numpy's abs_l0 @ beta), and
            // the argmin over them (its own fp64 keys)
            auto argmin_exact = [&]() {
                bk = ~0ULL;
                bj = 0x7fffffff;
#pragma unroll 1
                for (int i = 0; i < NC; ++i) {
                    const int j = p + G * i;
                    double qx = 0.0;
#pragma unroll 1
                    for (int k = 0; k < K; ++k) qx = qx + fabs(Af[Q.info_set[k]]) * Q.beta[k * K + j];
                    const uint64_t key = seen_j(j) ? ~0ULL : flip_order_key(qx);
                    if (key < bk) {
                        bk = key;
                        bj = j;
                    }
                }
#pragma unroll
                for (int sft = 1; sft < G; sft <<= 1) {
                    const uint64_t ok = shfl_u64(bk, lane ^ sft);
                    const int oj = __shfl(bj, lane ^ sft);
                    if (ok < bk || (ok == bk && oj < bj)) {
                        bk = ok;
                        bj = oj;
                    }
                }
            };
            if (Q.beta) {
                typedef float f2 __attribute__((ext_vector_type(2)));
                // candidates in blocks of 8 (L = 4: two passes over k), each k's |L0| read from the
                // leaves: fewer accumulators and loads in flight (registers, see the replay)
                constexpr int CB = NC < 8 ? NC : 8;
                const f2* bg = reinterpret_cast<const f2*>(P.fp_beta32g) + p * (NC / 2);
#pragma unroll
                for (int cb = 0; cb < NC / CB; ++cb) {
                    f2 acc[CB / 2];
#pragma unroll
                    for (int i = 0; i < CB / 2; ++i) acc[i] = (f2){0.0f, 0.0f};
#pragma unroll 2
                    for (int k = 0; k < K; ++k) {
                        const double ad = fabs(Af[Q.info_set[k]]);
                        if (cb == 0) as = as + ad;
                        const float a32 = (float)ad;
#pragma unroll
                        for (int i = 0; i < CB / 2; ++i)
                            acc[i] = __builtin_elementwise_fma((f2){a32, a32}, bg[k * G * (NC / 2) + cb * (CB / 2) + i], acc[i]);
                    }
#pragma unroll
                    for (int i = 0; i < CB / 2; ++i) {
                        qv[cb * CB + 2 * i] = acc[i].x;
                        qv[cb * CB + 2 * i + 1] = acc[i].y;
                    }
                }
                argmin();
                // dl_post_kernel's certificate of the packed fp32 sums (dlscl.hip): every other untried
                // candidate's sum above the best one's by twice the error bound, else the exact sums
                const double gk = (4.0 * (double)K + 8.0) * 0x1p-53;
                const double e2 = (as < 0x1p100 && as * Q.beta_absmax < 0x1p100)
                                      ? 2.04 * (as * Q.beta_absmax * (((double)K + 2.01) * 0x1p-24 + 0.5 * gk)
                                                + (double)K * 0x1p-149 + as * 0x1p-150 + (double)K * Q.beta_absmax * 0x1p-150)
                                      : __builtin_inf();
                double qmine = qv[0];
#pragma unroll
                for (int i = 1; i < NC; ++i) qmine = (bj >> LOG_G) == i ? (double)qv[i] : qmine;
                const double qb = pscl_asf64(shfl_u64(pscl_asu64(qmine), lane_lo + (bj & (G - 1))));
                const double thr = qb + e2 * (1.0 + 0x1p-40);
                bool near = false;
#pragma unroll
                for (int i = 0; i < NC; ++i) {
                    const int j = p + G * i;
                    near = near || (j != bj && !seen_j(j) && !((double)qv[i] > thr));
                }
                const bool fnear = frame_bits(wmask(near)) != 0;
                if (wmask(fnear && more) != 0) {
                    const int bj0 = bj;
                    argmin_exact();
                    if (!(fnear && more)) bj = bj0;  // (frames whose certificate held keep theirs)
                }
            } else {
                // (|L0| itself: argmin over the fp64 values, flip.py:107)
                bk = ~0ULL;
                bj = 0x7fffffff;
#pragma unroll 1
                for (int i = 0; i < NC; ++i) {
                    const int j = p + G * i;
                    const uint64_t key = seen_j(j) ? ~0ULL : flip_order_key(fabs(Af[Q.info_set[j]]));
                    if (key < bk) {
                        bk = key;
                        bj = j;
                    }
                }
#pragma unroll
                for (int sft = 1; sft < G; sft <<= 1) {
                    const uint64_t ok = shfl_u64(bk, lane ^ sft);
                    const int oj = __shfl(bj, lane ^ sft);
                    if (ok < bk || (ok == bk && oj < bj)) {
                        bk = ok;
                        bj = oj;
                    }
                }
            }
            const int idx = bj;  // (frame-uniform) an untried index exists: rounds <= min(retries, K)
            int seg = Q.info_set[idx < K ? idx : 0] >> 4;
            if (seg > PSCL_DL_NSEG - 1) seg = PSCL_DL_NSEG - 1;
            // ---- warm state: the forced prefix's metric at each 16-phase boundary, from the screening
            // tail (this kernel's own increments: good child + L, bad child + |lam| + L)
            double bs[PSCL_DL_NSEG];
#pragma unroll
            for (int b = 0; b < PSCL_DL_NSEG; ++b) {  // block b: the lane's phases q = p + G j in [16 b, 16 b + 16)
                double acc_b = 0.0;
#pragma unroll
                for (int jj = 0; jj < 16 / G; ++jj) {
                    const int q = p + G * (b * (16 / G) + jj);
                    const double lam = Af[q];
                    const uint32_t ubit = (uint32_t)(((q >> 6) ? bu1 : bu0) >> (q & 63)) & 1u;
                    const double Lt = pscl_softplus_tail_abs(lam);
                    const bool good = ubit == sign_bit(lam);
                    acc_b = acc_b + (good ? Lt : fabs(lam) + Lt);
                }
                bs[b] = acc_b;
            }
#pragma unroll
            for (int b = 0; b < PSCL_DL_NSEG; ++b)
#pragma unroll
                for (int sft = 1; sft < G; sft <<= 1) bs[b] = bs[b] + pscl_asf64(shfl_u64(pscl_asu64(bs[b]), lane ^ sft));
            if (more && p == 0) {
                double mt = 0.0;
                double* wm = Q.warm_metric + e * PSCL_DL_NSEG;
#pragma unroll
                for (int k = 0; k < PSCL_DL_NSEG; ++k) {
                    if (k <= seg) wm[k] = mt;
                    mt = mt + bs[k];
                }
                Q.warm_u[2 * e] = bu0;
                Q.warm_u[2 * e + 1] = bu1;
                Q.tried[2 * e] = idx < 64 ? (t0 | (1ULL << idx)) : t0;
                Q.tried[2 * e + 1] = idx >= 64 ? (t1 | (1ULL << (idx - 64))) : t1;
                Q.ntried[e] = nt + 1;
                if (Q.tried_out) Q.tried_out[x_frow * Q.tried_stride + nt] = idx;
                // _force_vector (flip.py:30-34): bits [0, idx) = reference, bit idx flipped, rest free
                uint64_t* fr = Q.force + e * 2 * PW;
#pragma unroll
                for (int w = 0; w < PW; ++w) {
                    const int lo = 64 * w, nb = idx - lo + 1;
                    const uint64_t mask = nb <= 0 ? 0ULL : (nb >= 64 ? ~0ULL : ((1ULL << nb) - 1ULL));
                    uint64_t val = (w ? bi1 : bi0) & mask;
                    if (idx >= lo && idx < lo + 64) val ^= 1ULL << (idx - lo);
                    fr[w] = mask;
                    fr[PW + w] = val;
                }
            }
            // ---- append to bucket seg of the next round: one atomic per (bucket, wavefront)
#pragma unroll
            for (int sg = 0; sg < PSCL_DL_NSEG; ++sg) {
                const uint64_t mm = wmask(more && p == 0 && seg == sg);
                if (mm == 0) continue;
                int base = 0;
                if (lane == (int)__builtin_ctzll(mm)) base = atomicAdd(Q.out_count + sg * PSCL_DL_CSTRIDE, __popcll(mm));
                base = __shfl(base, (int)__builtin_ctzll(mm));
                if ((mm >> lane) & 1ULL)
                    Q.out_list[(int64_t)sg * Q.cap + base + __popcll(mm & ((1ULL << lane) - 1ULL))] = (int32_t)e;
            }
            wave_lds_fence();  // (the next frame's decode rewrites the region)
        };
        // fused TX: the message words formed again for the epilogue from an opaque copy of the frame
        // counter -- left to itself the compiler reuses the frame start's draws and keeps them live
        // across the whole decode (with the rows' draws: +75 VGPRs, 2 waves/SIMD instead of 3)
        uint64_t tfr2 = tfr;
        if constexpr (TXF) {
            asm volatile("" : "+v"(tfr2));
            tx_frame_words(P, tfr2, tm, traw, tx);
        }
        // ---- epilogue: candidates u[info_set], CRC syndrome, final list order certified,
        // best = first CRC pass in list order (scl.py:176-209)
        uint64_t ib0 = 0, ib1 = 0;
        {
            int off = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t byte = (uint32_t)(((k < 8 ? u0 : u1) >> (8 * (k & 7))) & 255u);
                const uint64_t cb = (PSCL_LANE_ABL & 8) ? (uint64_t)byte : GT[k * 256 + byte];
                if (off < 64) {
                    ib0 |= cb << off;
                    if (off > 56) ib1 |= cb >> (64 - off);
                } else {
                    ib1 |= cb << (off - 64);
                }
                off += __builtin_popcount((uint32_t)(((k < 8 ? info0 : info1) >> (8 * (k & 7))) & 255u));
            }
        }
        uint32_t syn = 0;
        if (P.has_crc) {
            constexpr int k4 = (K + 3) >> 2;
#pragma unroll
            for (int m = 0; m < k4; ++m)
                syn ^= (PSCL_LANE_ABL & 8) ? (uint32_t)(((m < 16 ? ib0 : ib1) >> (4 * (m & 15))) & 15u) << m
                                           : ST[m * 16 + (uint32_t)(((m < 16 ? ib0 : ib1) >> (4 * (m & 15))) & 15u)];
        }
        // list position = rank of the metric among the frame's L (high words); certified when all
        // pairs are apart by the margin (then the ranks are distinct and equal the exact order).
        // FS: among the frame's live paths (lanes p < 2^lcnt; the others' keys above every metric)
        const bool live = !FS || p < (1 << lcnt);
        const uint32_t kh = live ? hiw(metric) : 0xffffffffu, ku = live ? hiw_up(metric) : 0xffffffffu;
        uint32_t r = 0;
        bool near = false;
        auto cmp_perm = [&](uint32_t oh, uint32_t ou) {
            r += oh < kh ? 1u : 0u;
            near = near || !(ku < oh || ou < kh);
        };
        if constexpr (EX) {
            r = (uint32_t)p;  // (the exact instance keeps list order in its lanes)
        } else {
            cmp_perm(dpp32<kQX1>(kh), dpp32<kQX1>(ku));
            cmp_perm(dpp32<kQX2>(kh), dpp32<kQX2>(ku));
            cmp_perm(dpp32<kQX3>(kh), dpp32<kQX3>(ku));
            if constexpr (G == 8) {
                const uint32_t mh = dpp32<kFMIR>(kh), mu = dpp32<kFMIR>(ku);
                cmp_perm(mh, mu);
                cmp_perm(dpp32<kQX1>(mh), dpp32<kQX1>(mu));
                cmp_perm(dpp32<kQX2>(mh), dpp32<kQX2>(mu));
                cmp_perm(dpp32<kQX3>(mh), dpp32<kQX3>(mu));
            }
        }
        amb |= wmask(near && live) & vmask;
        const bool famb = frame_bits(amb) != 0;
        if (famb && p == 0 && fvalid) {
            if constexpr (FS) {  // DL-SCL retry round: into the entry's deferred bucket (with the
                                 // fused post pass bucket 0: its warm metric is a screening one)
                const int fseg = (FP || P.warm_apx) ? 0 : pscl_bucket_of(fsafe, bpre);
                const int slot = atomicAdd(P.amb_count + fseg * PSCL_DL_CSTRIDE, 1);
                P.amb_elist[(int64_t)fseg * P.bcap + slot] = (int32_t)f;
                P.flags[f] = PSCL_DL_DEFERRED;
            } else {
                P.amb_list[atomicAdd(P.amb_count, 1)] = fi;
            }
        }
        // best: the lowest list position whose candidate passes the CRC (position 0 if none)
        const uint32_t pass = P.has_crc ? (syn == 0 ? 1u : 0u) : 1u;
        const uint32_t keyb = live ? (pass ? r : (uint32_t)LMAX + r) : 0xffffu;
        const uint32_t kbest = frame_min<G>(keyb);
        if (fvalid && !famb && keyb == kbest) {
            const int best = (int)(kbest & (uint32_t)(LMAX - 1));
            const bool bpass = kbest < (uint32_t)LMAX;
            const int64_t fo = (EX && !FS && P.out_by_row) ? frow : f;  // (the re-decode: at the frame's row)
            if (P.best) {
                P.best[fo * PW] = ib0;
                if (PW > 1) P.best[fo * PW + 1] = ib1;
            }
            if (P.flags) P.flags[fo] = (uint8_t)((bpass ? PSCL_FLAG_CRC_PASS : 0u) | (uint32_t)best);
            if (P.n_paths) P.n_paths[fo] = FS ? (1 << lcnt) : LMAX;
            if (!FS && P.ref) {
                const uint64_t ibw[2] = {ib0, ib1};
                tally_errors(ibw, TXF ? tm : P.ref + fo * PW, PW, P.k_payload, bpass, cfe, cbe, cpe, cpb);
            }
        }
        if constexpr (FS) {
            if constexpr (FP) fused_post(famb, live, keyb, kbest, ib0, ib1, u0, u1, frow, f, fvalid);
        }
        if constexpr (TXF) {
            // the message words of every frame (the counts' reference; the rows of the frames the exact
            // re-decode or the retry chain will read are written by tx_rows_kernel, scl_kernels.hip)
            if (fvalid && p == 0) {
                P.tx_msg[fi * PW] = tm[0];
                if (PW > 1) P.tx_msg[fi * PW + 1] = tm[1];
            }
        }
        wave_lds_fence();
    }
    if (!FS && P.ref) {
        flush_counts_p(P, blockIdx.x, cfe, cbe, cpe, cpb);
        if (blockIdx.x == 0 && threadIdx.x == 0 && !(EX && P.out_by_row))  // (a re-decode's frames were counted)
            atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + PSCL_CNT_FRAMES, (unsigned long long)P.B);
    }
    if constexpr (FS) {
        if (FP && P.fp.counters && __builtin_amdgcn_ballot_w64(pdecodes != 0)) {
            const int d = wave_sum(pdecodes);
            if (lane == 0) atomicAdd(reinterpret_cast<unsigned long long*>(P.fp.counters) + PSCL_CNT_RETRIES, (unsigned long long)d);
        }
    }
    if constexpr (TXF) {
        if (P.tx_upart && __builtin_amdgcn_ballot_w64((tufe | tube) != 0)) {
            const int fe = wave_sum(tufe), be = wave_sum(tube);
            if (lane == 0) reinterpret_cast<int4*>(P.tx_upart)[blockIdx.x] = make_int4(fe, be, 0, 0);
        }
        if (P.tx_unc_counters && blockIdx.x == 0 && threadIdx.x == 0)
            atomicAdd(reinterpret_cast<unsigned long long*>(P.tx_unc_counters) + PSCL_CNT_FRAMES, (unsigned long long)P.B);
    }
}

}  // namespace

// the lane-per-path screening launch of a plain (128,64) decode at L = 4 or 8: one wavefront of
// 64 / L frames per workgroup, LDS = 30 L doubles per frame (15 KB per workgroup at both sizes)
int pscl_lane_frames_per_wg(int L) { return 64 / L; }

// timing-only: unused LDS bytes added to each plain launch (occupancy experiments; 0 in the product)
#ifndef PSCL_LANE_LDS_PAD
#define PSCL_LANE_LDS_PAD 0
#endif

hipError_t pscl_launch_lane(const pscl_decode_params& P, int64_t grid, hipStream_t s) {
    // (pscl_lane_available: the (128,64) code on plain rows, or the rate-matched NR (128,88) code)
    const int lds8 = LaneLayout<8>::F * LaneLayout<8>::FSTRIDE * 8 + PSCL_LANE_LDS_PAD,
              lds4 = LaneLayout<4>::F * LaneLayout<4>::FSTRIDE * 8 + PSCL_LANE_LDS_PAD;
    if (P.tx) {  // the fused TX instance (plain rows of the (128,64) code, pscl_simulate_device)
        if (P.rm_E) return hipErrorInvalidValue;
        if (P.L == 8)
            hipLaunchKernelGGL((scl_lane_kernel<8, 1, false, true>), dim3((unsigned)grid), dim3(64), lds8, s, P);
        else if (P.L == 4)
            hipLaunchKernelGGL((scl_lane_kernel<4, 1, false, true>), dim3((unsigned)grid), dim3(64), lds4, s, P);
        else
            return hipErrorInvalidValue;
        return hipGetLastError();
    }
    if (P.L == 8 && !P.rm_E)
        hipLaunchKernelGGL((scl_lane_kernel<8, 1>), dim3((unsigned)grid), dim3(64), lds8, s, P);
    else if (P.L == 8)
        hipLaunchKernelGGL((scl_lane_kernel<8, 2>), dim3((unsigned)grid), dim3(64), lds8, s, P);
    else if (P.L == 4 && !P.rm_E)
        hipLaunchKernelGGL((scl_lane_kernel<4, 1>), dim3((unsigned)grid), dim3(64), lds4, s, P);
    else if (P.L == 4)
        hipLaunchKernelGGL((scl_lane_kernel<4, 2>), dim3((unsigned)grid), dim3(64), lds4, s, P);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// the exact lane-per-path launch (pscl_lane_exact_available): the deferred frames' re-decode of a
// plain decode, or an exact forced-bit retry round (FS); grid capped by P.grid_cap
int64_t pscl_lane_exact_grid(const pscl_decode_params& P) {
    const int F = 64 / P.L;
    const int64_t grid = (P.B + F - 1) / F, cap = P.grid_cap > 0 ? P.grid_cap : (1 << 20);
    return grid < 1 ? 1 : (grid > cap ? cap : grid);
}

hipError_t pscl_launch_lane_exact(const pscl_decode_params& P, hipStream_t s) {
    const int64_t grid = pscl_lane_exact_grid(P);
    const int lds8 = LaneLayout<8>::F * LaneLayout<8>::FSTRIDE_EX * 8, lds4 = LaneLayout<4>::F * LaneLayout<4>::FSTRIDE_EX * 8;
    const dim3 g((unsigned)grid), b(64);
    if (P.force) {
        if (P.L == 8)
            hipLaunchKernelGGL((scl_lane_kernel<8, 1, true, false, false, true>), g, b, lds8, s, P);
        else if (P.L == 4)
            hipLaunchKernelGGL((scl_lane_kernel<4, 1, true, false, false, true>), g, b, lds4, s, P);
        else
            return hipErrorInvalidValue;
    } else if (P.L == 8) {
        if (P.rm_E)
            hipLaunchKernelGGL((scl_lane_kernel<8, 2, false, false, false, true>), g, b, lds8, s, P);
        else
            hipLaunchKernelGGL((scl_lane_kernel<8, 1, false, false, false, true>), g, b, lds8, s, P);
    } else if (P.L == 4) {
        if (P.rm_E)
            hipLaunchKernelGGL((scl_lane_kernel<4, 2, false, false, false, true>), g, b, lds4, s, P);
        else
            hipLaunchKernelGGL((scl_lane_kernel<4, 1, false, false, false, true>), g, b, lds4, s, P);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// the lane-per-path forced-bit screening launch of a DL-SCL retry round (pscl_lane_fs_available)
hipError_t pscl_launch_lane_fs(const pscl_decode_params& P, int64_t grid, hipStream_t s) {
    const int lds8 = LaneLayout<8>::F * (P.fpost ? LaneLayout<8>::FSTRIDE_FS : LaneLayout<8>::FSTRIDE) * 8,
              lds4 = LaneLayout<4>::F * (P.fpost ? LaneLayout<4>::FSTRIDE_FS : LaneLayout<4>::FSTRIDE) * 8;
    if (P.fpost && (P.K != 64 || (P.fp.beta && !P.fp_beta32g))) return hipErrorInvalidValue;
    if (P.L == 8)
        if (P.fpost)
            hipLaunchKernelGGL((scl_lane_kernel<8, 1, true, false, true>), dim3((unsigned)grid), dim3(64), lds8, s, P);
        else
            hipLaunchKernelGGL((scl_lane_kernel<8, 1, true>), dim3((unsigned)grid), dim3(64), lds8, s, P);
    else if (P.L == 4)
        if (P.fpost)
            hipLaunchKernelGGL((scl_lane_kernel<4, 1, true, false, true>), dim3((unsigned)grid), dim3(64), lds4, s, P);
        else
            hipLaunchKernelGGL((scl_lane_kernel<4, 1, true>), dim3((unsigned)grid), dim3(64), lds4, s, P);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}
