// scl_device.h -- device helpers shared by the decode kernels (wavefront = 64 lanes).
#ifndef PSCL_SCL_DEVICE_H
#define PSCL_SCL_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "glibc_softplus.h"
#include "polar_scl.h"

// Timing-only ablation switches for diagnostic builds (tools/ablate.py); 0 in the product.
#ifndef PSCL_ABLATE
#define PSCL_ABLATE 0
#endif

namespace pscl {

constexpr int kWave = 64;

__device__ __forceinline__ uint32_t bperm32(uint32_t v, int src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    uint32_t lo = bperm32((uint32_t)v, src), hi = bperm32((uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ double shfl_f64(double v, int src) {
    return pscl_asf64(shfl_u64(pscl_asu64(v), src));
}
__device__ __forceinline__ uint32_t rdl_u32(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ double rdl_f64(double v, int l) {
    uint64_t u = pscl_asu64(v);
    uint32_t lo = rdl_u32((uint32_t)u, l), hi = rdl_u32((uint32_t)(u >> 32), l);
    return pscl_asf64(((uint64_t)hi << 32) | lo);
}

// Orders the wave's LDS traffic: hardware executes one wave's LDS instructions in order;
// this keeps the compiler from moving loads above the stores they depend on.
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef PSCL_F_ASM
#define PSCL_F_ASM 1
#endif
// f(a,b) = sign(a) sign(b) min(|a|,|b|)  (polar.py:122-123).  Exact: the result is one of the
// inputs' magnitudes with the XOR of the signs (sign(0) = 0 makes a +-0 result either way, and
// the sign of a zero never reaches a decision or a metric).  v_min_f64 with |.| source
// modifiers (written out: fmin would add two canonicalising v_max_f64 for signalling NaNs,
// which finite LLRs never are) + v_xor + v_and_or.
__device__ __forceinline__ double f_minsum(double a, double b) {
    double m;
    asm("v_min_f64 %0, |%1|, |%2|" : "=v"(m) : "v"(a), "v"(b));
    const uint64_t ab = pscl_asu64(a), bb = pscl_asu64(b), mb = pscl_asu64(m);
    const uint32_t x = (uint32_t)(ab >> 32) ^ (uint32_t)(bb >> 32);
#if PSCL_F_ASM
    // v_and_or_b32 with the sign mask in an SGPR: a VOP3 encoding takes no literal on gfx950, and
    // left to itself the compiler splits the fold into v_and_b32 (literal) + v_or_b32
    uint32_t hi;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(hi) : "v"(x), "s"(0x80000000u), "v"((uint32_t)(mb >> 32)));
#else
    const uint32_t hi = (uint32_t)(mb >> 32) | (x & 0x80000000u);
#endif
    return pscl_asf64(((uint64_t)hi << 32) | (uint32_t)mb);
}
// g(a,b,c) = b + (1-2c) a  (polar.py:126-127): b + (+-a), one rounding, sign of a flipped by c
__device__ __forceinline__ double g_node(double a, double b, uint32_t c) {
    const uint64_t ab = pscl_asu64(a);
    const uint32_t hi = (uint32_t)(ab >> 32) ^ (c << 31);
    return b + pscl_asf64(((uint64_t)hi << 32) | (uint32_t)ab);
}

// g(a, b, c) with c = bit `pos` of the 32-bit word w (pos may differ per lane): the bit is
// moved to bit 31 and folded into a's sign in one v_bitop3 (a ^ (m & 0x80000000)); no 64-bit
// shift of the partial-sum word
__device__ __forceinline__ double g_node_wbit(double a, double b, uint32_t w, uint32_t pos) {
    const uint64_t ab = pscl_asu64(a);
    const uint32_t hi = (uint32_t)(ab >> 32) ^ ((w << (31u - pos)) & 0x80000000u);
    return b + pscl_asf64(((uint64_t)hi << 32) | (uint32_t)ab);
}

// g(a, b, c) with c = bit 31 of w (the bit already moved there, e.g. by a 64-bit shift serving two
// nodes): a's sign ^= w & 0x80000000 in one v_bitop3 (written out: the compiler splits it into
// v_and + v_xor once the shift is not part of the pattern)
__device__ __forceinline__ double g_node_bit31(double a, double b, uint32_t w) {
    const uint64_t ab = pscl_asu64(a);
    uint32_t hi;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6c" : "=v"(hi) : "v"(w), "v"((uint32_t)(ab >> 32)), "s"(0x80000000u));
    return b + pscl_asf64(((uint64_t)hi << 32) | (uint32_t)ab);
}

// max(-v, 0): the part of np.logaddexp(0, -v) beyond the shared tail (bit 0 pays |v| when
// v < 0); one v_max_f64 with the negation as a source modifier (fmax would canonicalise)
__device__ __forceinline__ double relu_neg(double v) {
    double d;
    asm("v_max_f64 %0, -%1, 0" : "=v"(d) : "v"(v));
    return d;
}

// bit 31 of the high word of v: 1 for negative v (and -0.0)
__device__ __forceinline__ uint32_t sign_bit(double v) { return (uint32_t)(pscl_asu64(v) >> 63); }

// Arikan transform of the low w bits of x (in-word, w <= 64): bit j ^= bit j+s for bit s of j
// clear, for every stage s (stages commute).  Bits >= w must be zero.
__device__ __forceinline__ uint64_t polar_transform64(uint64_t x) {
    x ^= (x >> 1) & 0x5555555555555555ULL;
    x ^= (x >> 2) & 0x3333333333333333ULL;
    x ^= (x >> 4) & 0x0f0f0f0f0f0f0f0fULL;
    x ^= (x >> 8) & 0x00ff00ff00ff00ffULL;
    x ^= (x >> 16) & 0x0000ffff0000ffffULL;
    x ^= (x >> 32) & 0x00000000ffffffffULL;
    return x;
}

// transform of a segment of at most 32 (resp. 16, 8) bits held in a 32-bit word
__device__ __forceinline__ uint32_t polar_transform32(uint32_t x) {
    x ^= (x >> 1) & 0x55555555u;
    x ^= (x >> 2) & 0x33333333u;
    x ^= (x >> 4) & 0x0f0f0f0fu;
    x ^= (x >> 8) & 0x00ff00ffu;
    x ^= (x >> 16) & 0x0000ffffu;
    return x;
}
__device__ __forceinline__ uint32_t polar_transform16(uint32_t x) {
    x ^= (x >> 1) & 0x5555u;
    x ^= (x >> 2) & 0x3333u;
    x ^= (x >> 4) & 0x0f0fu;
    x ^= (x >> 8) & 0x00ffu;
    return x;
}
__device__ __forceinline__ uint32_t polar_transform8(uint32_t x) {
    x ^= (x >> 1) & 0x55u;
    x ^= (x >> 2) & 0x33u;
    x ^= (x >> 4) & 0x0fu;
    return x;
}

// metric increments of both bit hypotheses, np.logaddexp(0, -+llr) (scl.py:102-105):
// max(0,v) + L with v = -llr (bit 0) / +llr (bit 1); L = log1p(exp(-|llr|)); llr == 0 -> LOGE2.
// The "bad" child pays |llr| + L (|llr| = -v exactly), the "good" one 0.0 + L = L.  An exactly
// zero LLR is a wave-uniform rare branch.
__device__ __forceinline__ void metric_incr(double lam, double L, double& i0, double& i1) {
    const double t = fabs(lam) + L;
    const bool neg = lam < 0.0;
    i0 = neg ? t : L;
    i1 = neg ? L : t;
    if (PSCL_RARE(lam == 0.0)) {
        const bool z = lam == 0.0;
        i0 = z ? PSCL_LOGE2 : i0;
        i1 = z ? PSCL_LOGE2 : i1;
    }
}

__device__ __forceinline__ uint64_t pick_word(uint64_t w0, uint64_t w1, int idx) { return idx ? w1 : w0; }


// ---------------------------------------------------------------- lane-group helpers
// A wavefront decodes F = 64/G frames at once; frame slot fl owns the G = 2*LMAX lanes
// [fl*G, fl*G + G).  Lane g < L of a group holds list path g (list position == lane, so the
// stable-sort tie key is the lane index itself); lanes [L, 2L) carry the bit-1 children
// while the list is being extended.

template <int G, int K>
__device__ __forceinline__ uint32_t grot32c(uint32_t v, int lane) {
    if constexpr (G == 16) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + K, 0xF, 0xF, true);  // row_ror:K
    } else if constexpr (G == 8) {
        const uint32_t a = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + K, 0xF, 0xF, true);
        const uint32_t b = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + K + 8, 0xF, 0xF, true);
        return ((lane & 7) >= K) ? a : b;  // row_ror:K reads lane x-K; wrap inside the 8-lane group
    } else if constexpr (G == 4) {
        constexpr int q = ((0 + K) & 3) | (((1 + K) & 3) << 2) | (((2 + K) & 3) << 4) | (((3 + K) & 3) << 6);
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, q, 0xF, 0xF, true);  // quad_perm
    } else if constexpr (G == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
    } else {
        return bperm32(v, (lane & ~(G - 1)) | ((lane + K) & (G - 1)));
    }
}

template <int G, int K>
__device__ __forceinline__ double grot64c(double v, int lane) {
    const uint64_t u = pscl_asu64(v);
    const uint32_t lo = grot32c<G, K>((uint32_t)u, lane), hi = grot32c<G, K>((uint32_t)(u >> 32), lane);
    return pscl_asf64(((uint64_t)hi << 32) | lo);
}

// Stable rank of this lane's key among the G keys of its group.  The key is (metric, t):
// metrics are sums of non-negative increments, never -0 or NaN, and +inf marks an empty
// candidate, so their IEEE bit patterns order like unsigned integers and the whole key
// compares as one 96-bit unsigned number (hi word, lo word, t) with a borrow chain.
// One rank rotation for 16-lane groups, hand-scheduled: the 96-bit subtract (lane g-K minus
// lane g) runs as three DPP-fused VOP2 subtracts chained through VCC, and the final borrow
// (= "that key is smaller") is added into r.  4 VALU, no SGPR masks.  The leading s_nop covers
// the VALU-write -> DPP-read hazard on the key registers (inline asm is not hazard-checked).
template <int K>
__device__ __forceinline__ void rank_rot16(uint32_t mh, uint32_t ml, uint32_t t, uint32_t& r) {
    uint32_t tmp;
    asm volatile(
        "s_nop 1\n\t"
        "v_sub_co_u32_dpp %0, vcc, %2, %2 row_ror:%5 row_mask:0xf bank_mask:0xf\n\t"
        "v_subb_co_u32_dpp %0, vcc, %3, %3, vcc row_ror:%5 row_mask:0xf bank_mask:0xf\n\t"
        "v_subb_co_u32_dpp %0, vcc, %4, %4, vcc row_ror:%5 row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32 %1, vcc, 0, %1, vcc"
        : "=&v"(tmp), "+v"(r)
        : "v"(t), "v"(ml), "v"(mh), "i"(K)
        : "vcc");
}

template <int G, int K>
__device__ __forceinline__ void rank_step(uint32_t mh, uint32_t ml, uint32_t t, int lane, uint32_t& r) {
    if constexpr (G == 16 && K < G) {
        rank_rot16<K>(mh, ml, t, r);
        rank_step<G, K + 1>(mh, ml, t, lane, r);
    } else if constexpr (K < G) {
        const uint32_t th = grot32c<G, K>(t, lane);
        const uint32_t lh = grot32c<G, K>(ml, lane);
        const uint32_t hh = grot32c<G, K>(mh, lane);
        unsigned c0, c1, c2;
        (void)__builtin_subc(th, t, 0u, &c0);
        (void)__builtin_subc(lh, ml, c0, &c1);
        (void)__builtin_subc(hh, mh, c1, &c2);
        r += c2;  // 1 iff key of lane (g-K) < my key
        rank_step<G, K + 1>(mh, ml, t, lane, r);
    }
}

// rank over rotations K = K0 .. KEND-1 only (keys duplicated so that fewer rotations cover
// every other key of interest)
template <int G, int K, int KEND>
__device__ __forceinline__ void rank_step_n(uint32_t mh, uint32_t ml, uint32_t t, int lane, uint32_t& r) {
    if constexpr (G == 16 && K < KEND) {
        rank_rot16<K>(mh, ml, t, r);
        rank_step_n<G, K + 1, KEND>(mh, ml, t, lane, r);
    } else if constexpr (K < KEND) {
        const uint32_t th = grot32c<G, K>(t, lane);
        const uint32_t lh = grot32c<G, K>(ml, lane);
        const uint32_t hh = grot32c<G, K>(mh, lane);
        unsigned c0, c1, c2;
        (void)__builtin_subc(th, t, 0u, &c0);
        (void)__builtin_subc(lh, ml, c0, &c1);
        (void)__builtin_subc(hh, mh, c1, &c2);
        r += c2;
        rank_step_n<G, K + 1, KEND>(mh, ml, t, lane, r);
    }
}

// Metric-only rank: the number of keys of the group (rotations K .. KEND-1) whose 64-bit
// metric is strictly smaller than this lane's.  Equals the stable rank whenever the metrics
// of the keys that matter are distinct; equal metrics give two lanes the same rank, which the
// callers detect (a list position nobody claims) and then redo with the full tie key.
// 3 VALU per rotation instead of 4.
template <int K>
__device__ __forceinline__ void rank_rot16_m(uint32_t mh, uint32_t ml, uint32_t& r) {
    uint32_t tmp;
    asm volatile(
        "s_nop 1\n\t"
        "v_sub_co_u32_dpp %0, vcc, %2, %2 row_ror:%4 row_mask:0xf bank_mask:0xf\n\t"
        "v_subb_co_u32_dpp %0, vcc, %3, %3, vcc row_ror:%4 row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32 %1, vcc, 0, %1, vcc"
        : "=&v"(tmp), "+v"(r)
        : "v"(ml), "v"(mh), "i"(K)
        : "vcc");
}

template <int G, int K, int KEND>
__device__ __forceinline__ void rank_step_m(uint32_t mh, uint32_t ml, int lane, uint32_t& r) {
    if constexpr (G == 16 && K < KEND) {
        rank_rot16_m<K>(mh, ml, r);
        rank_step_m<G, K + 1, KEND>(mh, ml, lane, r);
    } else if constexpr (K < KEND) {
        const uint32_t lh = grot32c<G, K>(ml, lane);
        const uint32_t hh = grot32c<G, K>(mh, lane);
        unsigned c1, c2;
        (void)__builtin_subc(lh, ml, 0u, &c1);
        (void)__builtin_subc(hh, mh, c1, &c2);
        r += c2;
        rank_step_m<G, K + 1, KEND>(mh, ml, lane, r);
    }
}

// Screening rank on 32-bit keys (the high words of the metrics): +1 for every key of the
// group, rotations K .. KEND-1, strictly below this lane's.  16-lane groups: one DPP-fused
// subtract (borrow = "that key is smaller") + one add-with-carry per rotation; FIRST carries
// the s_nop that covers a VALU write of the key just before (inline asm is not hazard-checked;
// the later rotations read the same, unchanged key register).
template <int K, bool FIRST>
__device__ __forceinline__ void rank_rot16_h(uint32_t h, uint32_t& r) {
    uint32_t tmp;
    if constexpr (FIRST)
        asm volatile(
            "s_nop 1\n\t"
            "v_sub_co_u32_dpp %0, vcc, %2, %2 row_ror:%3 row_mask:0xf bank_mask:0xf\n\t"
            "v_addc_co_u32 %1, vcc, 0, %1, vcc"
            : "=&v"(tmp), "+v"(r)
            : "v"(h), "i"(K)
            : "vcc");
    else
        asm volatile(
            "v_sub_co_u32_dpp %0, vcc, %2, %2 row_ror:%3 row_mask:0xf bank_mask:0xf\n\t"
            "v_addc_co_u32 %1, vcc, 0, %1, vcc"
            : "=&v"(tmp), "+v"(r)
            : "v"(h), "i"(K)
            : "vcc");
}

template <int G, int K, int KEND>
__device__ __forceinline__ void rank_step_h(uint32_t h, int lane, uint32_t& r) {
    if constexpr (G == 16 && K < KEND) {
        rank_rot16_h<K, K == 1>(h, r);
        rank_step_h<G, K + 1, KEND>(h, lane, r);
    } else if constexpr (K < KEND) {
        const uint32_t o = grot32c<G, K>(h, lane);
        r += o < h ? 1u : 0u;
        rank_step_h<G, K + 1, KEND>(h, lane, r);
    }
}

// value of lane - 1 within each 16-lane row (row_shr:1; lane 0 of a row reads 0).  A plain
// DPP move in inline asm: left to the compiler, the move is folded into the consumer
// (v_subrev_u32_dpp of the very next instruction), which measured wrong on gfx950 right
// after the ds_bpermute that produces v (every frame flagged ambiguous).  The s_nop covers a
// VALU write of v just before (inline asm is not hazard-checked).
__device__ __forceinline__ uint32_t prev_lane32(uint32_t v) {
    uint32_t d;
    asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(d) : "v"(v));
    return d;
}

// OR of v over the G lanes of the group
template <int G, int K = 1>
__device__ __forceinline__ uint32_t or_reduce_group(uint32_t v, int lane, uint32_t acc = 0) {
    if constexpr (K == 1) acc = v;
    if constexpr (K < G) {
        acc |= grot32c<G, K>(v, lane);
        return or_reduce_group<G, K + 1>(v, lane, acc);
    } else {
        return acc;
    }
}

// value from lane g - LMAX of the group (the bit-0 sibling of a bit-1 candidate lane)
template <int G, int LMAX>
__device__ __forceinline__ uint32_t from_lower_half(uint32_t v, int lane) {
    if constexpr (G <= 16) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + LMAX, 0xF, 0xF, true);  // row_ror:LMAX
    } else {
        return bperm32(v, lane - LMAX);
    }
}


// value from lane g + LMAX of the group (the bit-1 half), G = 2*LMAX <= 16
template <int G, int LMAX>
__device__ __forceinline__ uint32_t from_upper_half(uint32_t v, int lane) {
    if constexpr (G <= 16) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + ((16 - LMAX) & 15), 0xF, 0xF, true);
    } else {
        return bperm32(v, lane + LMAX);
    }
}

// Lanes g >= LMAX of the group take `up` from lane g - LMAX, lanes g < LMAX keep `own`:
// `path_lane ? own : from_lower_half(up)` as one DPP move whose bank mask leaves the lower
// half unwritten (its old value is `own`).  G = 16: the upper half is banks 2, 3 of the row;
// G = 8: banks 1, 3 (row_ror:4 stays inside the 8-lane group for those lanes).
template <int G, int LMAX>
__device__ __forceinline__ uint32_t merge_from_lower(uint32_t own, uint32_t up, int lane) {
    if constexpr (G == 16) {
        return (uint32_t)__builtin_amdgcn_update_dpp((int)own, (int)up, 0x128, 0xF, 0xC, false);
    } else if constexpr (G == 8) {
        return (uint32_t)__builtin_amdgcn_update_dpp((int)own, (int)up, 0x124, 0xF, 0xA, false);
    } else {
        const uint32_t x = from_lower_half<G, LMAX>(up, lane);
        return (lane & (G - 1)) < LMAX ? own : x;
    }
}

template <int G, int LMAX>
__device__ __forceinline__ uint64_t merge_from_lower64(uint64_t own, uint64_t up, int lane) {
    return ((uint64_t)merge_from_lower<G, LMAX>((uint32_t)(own >> 32), (uint32_t)(up >> 32), lane) << 32) |
           merge_from_lower<G, LMAX>((uint32_t)own, (uint32_t)up, lane);
}

// Wave masks of lane-position predicates: bits [0, n) of every G-lane group.
template <int G>
__device__ __forceinline__ constexpr uint64_t group_rep() {
    uint64_t m = 0;
    for (int k = 0; k < 64; k += G) m |= 1ULL << k;
    return m;
}
template <int G>
__device__ __forceinline__ constexpr uint64_t group_prefix_mask(int n) {
    return (n >= G ? ((G == 64) ? ~0ULL : ((1ULL << G) - 1)) : ((1ULL << n) - 1)) * group_rep<G>();
}
__device__ __forceinline__ uint64_t wmask(bool c) { return __builtin_amdgcn_ballot_w64(c); }

template <int G, int LMAX>
__device__ __forceinline__ uint64_t from_lower_half64(uint64_t v, int lane) {
    return ((uint64_t)from_lower_half<G, LMAX>((uint32_t)(v >> 32), lane) << 32) |
           from_lower_half<G, LMAX>((uint32_t)v, lane);
}

template <int G, int LMAX>
__device__ __forceinline__ uint64_t from_upper_half64(uint64_t v, int lane) {
    return ((uint64_t)from_upper_half<G, LMAX>((uint32_t)(v >> 32), lane) << 32) |
           from_upper_half<G, LMAX>((uint32_t)v, lane);
}

// Internal LLR i of an NR rate-matched frame (nr/polar/scl_nr.py:47-48): de-rate-match
// (rate_match.py:19-39: repeats averaged in numpy's order, E <= N padded with -1.0) then
// sub-block de-interleave (interleaver.py:26-37), as one gather from the E received LLRs.
__device__ __forceinline__ double nr_stage(const double* src, int k, int E, int N) {
    if (E <= N) return k < E ? src[k] : -1.0;
    const int reps = E / N, rem = E - reps * N;
    double s = src[k];
    for (int r = 1; r < reps; ++r) s = s + src[k + r * N];
    s = 0.0 + s;
    int cnt = reps;
    if (k < rem) {
        s = s + src[reps * N + k];
        ++cnt;
    }
    return s / (double)cnt;
}

// error counters of one decoded frame (run_fer_sweep.py:91-109, run_ber_sweep.py:77-82,156)
// value of lane - 1 within each 16-lane row (row_shr:1; lane 0 of a row reads 0)
__device__ __forceinline__ uint64_t prev_lane64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, 0x111, 0xF, 0xF, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), 0x111, 0xF, 0xF, true);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s);
    return v;
}

__device__ __forceinline__ void count_errors(int64_t* counters, uint64_t ib0, uint64_t ib1, uint64_t r0, uint64_t r1,
                                             int k_payload, bool pass) {
    const uint64_t d0 = ib0 ^ r0, d1 = ib1 ^ r1;
    const int bit_err = __popcll(d0) + __popcll(d1);
    const int kp = k_payload;
    const uint64_t pm0 = kp >= 64 ? ~0ULL : ((1ULL << kp) - 1);
    const uint64_t pm1 = kp >= 128 ? ~0ULL : (kp > 64 ? ((1ULL << (kp - 64)) - 1) : 0ULL);
    const int pay_err = __popcll(d0 & pm0) + __popcll(d1 & pm1);
    unsigned long long* C = reinterpret_cast<unsigned long long*>(counters);
    if (!pass) atomicAdd(C + PSCL_CNT_FRAME_ERR, 1ULL);
    if (bit_err) atomicAdd(C + PSCL_CNT_BIT_ERR, (unsigned long long)bit_err);
    if (pay_err) {
        atomicAdd(C + PSCL_CNT_PAYLOAD_ERR, 1ULL);
        atomicAdd(C + PSCL_CNT_PAYLOAD_BIT, (unsigned long long)pay_err);
    }
}

// FER/BER counters of a wavefront's frames (counts per lane, any lanes), added with one atomic per
// counter and wavefront: per-frame atomics on the four counter words serialise at the L2 (~10 ns
// each on one address; 10^5 failing frames per 10^6 at 4 dB)
__device__ __forceinline__ void flush_counts(int64_t* counters, int fe, int be, int pe, int pb) {
    fe = wave_sum(fe);
    be = wave_sum(be);
    pe = wave_sum(pe);
    pb = wave_sum(pb);
    if ((threadIdx.x & 63) == 0) {
        unsigned long long* C = reinterpret_cast<unsigned long long*>(counters);
        if (fe) atomicAdd(C + PSCL_CNT_FRAME_ERR, (unsigned long long)fe);
        if (be) atomicAdd(C + PSCL_CNT_BIT_ERR, (unsigned long long)be);
        if (pe) atomicAdd(C + PSCL_CNT_PAYLOAD_ERR, (unsigned long long)pe);
        if (pb) atomicAdd(C + PSCL_CNT_PAYLOAD_BIT, (unsigned long long)pb);
    }
}

// errors of one decoded frame against its reference words (count_errors' quantities), added to
// the lane's running counts
__device__ __forceinline__ void tally_errors(const uint64_t* ib, const uint64_t* ref, int W, int k_payload, bool pass,
                                             int& fe, int& be, int& pe, int& pb) {
    int bit_err = 0, pay_err = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {  // (unrolled: callers with a compile-time W keep ib in registers)
        const uint64_t dff = ib[w] ^ ref[w];
        const int kp = k_payload - 64 * w;
        const uint64_t pm = kp >= 64 ? ~0ULL : (kp > 0 ? ((1ULL << kp) - 1) : 0ULL);
        bit_err += __popcll(dff);
        pay_err += __popcll(dff & pm);
    }
    fe += pass ? 0 : 1;
    be += bit_err;
    pe += pay_err ? 1 : 0;
    pb += pay_err;
}

// ---- the TX stream (channel_kernel, scl_kernels.hip; the fused-TX lane kernel, scl128_lane.hip)

struct u32x4 {
    uint32_t x, y, z, w;
};

// Philox4x32-10 (Salmon et al., SC'11)
__device__ __forceinline__ u32x4 philox4x32(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        c = u32x4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// Box-Muller pair from one Philox block (a, bb): u1 in (0, 1] from the top 53 bits of a, u2 in
// [0, 1) from the top 24 bits of bb; radius and angle with the fp32 hardware transcendentals
// (v_log_f32, v_sqrt_f32, v_sin/cos_f32 in revolutions), the pair widened to fp64.  u1 keeps
// all 53 bits (its fp32 image is normal down to 2^-53), so the tail reaches 8.57 sigma like an
// fp64 draw; the fp32 roundings perturb a normal by ~1e-6 sigma, far below Monte-Carlo error
// (tests/test_gpu_channel.py states the tolerance).  One fp64 log and sincospi per pair took
// most of the TX kernel's time.
__device__ __forceinline__ void bm_pair(uint64_t a, uint64_t bb, double& z0, double& z1) {
    const float u1 = (float)(((double)(a >> 11) + 1.0) * 0x1p-53);
    const float u2 = (float)(uint32_t)(bb >> 40) * 0x1p-24f;
    const float rad = __builtin_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));  // -2 ln u1
    z0 = (double)(rad * __builtin_amdgcn_cosf(u2));
    z1 = (double)(rad * __builtin_amdgcn_sinf(u2));
}

}  // namespace pscl

#endif
