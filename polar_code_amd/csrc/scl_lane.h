// scl_lane.h -- cross-lane helpers of the lane-per-path screening decoders (scl128_lane.hip,
// scl_lane_long.hip): one lane per list path, G = L lanes per frame, DPP within a frame's lanes.
#ifndef PSCL_SCL_LANE_H
#define PSCL_SCL_LANE_H

#include "scl128_impl.h"

// the one-swap tier between the keep-the-better-children path and the full ranking
#ifndef PSCL_LANE_SWAP
#define PSCL_LANE_SWAP 1
#endif


// plain decodes compute the LLR tree in units of log2 e and the metrics in bits (the tail without its
// two fp32 multiplies, glibc_softplus.h pscl_softplus_tail2); the N = 128 FS retry decodes, whose
// warm-start metrics come from the post pass in nats, keep the natural-log form
#ifndef PSCL_LANE_BITS
#define PSCL_LANE_BITS 1
#endif

namespace {

// intra-frame lane permutations of an 8-lane group (DPP controls): quad_perm xor 1, 2, 3, and the
// half-row mirror (lane i <-> 7 - i), which maps one quad onto the other
constexpr int kQX1 = 0xB1, kQX2 = 0x4E, kQX3 = 0x1B, kQID = 0xE4, kHMIR = 0x141;
// the permutation that maps one quad of an 8-lane frame onto the other: row_half_mirror (0x141,
// lane i <-> 7 - i) for frames of 8 consecutive lanes; row_mirror (0x140, lane i <-> 15 - i) for the
// N = 128 kernel's frames of the outer or the inner two quads of a row (scl128_lane.hip)
#ifndef PSCL_LANE_FRAME_MIRROR
#define PSCL_LANE_FRAME_MIRROR 0x141
#endif
constexpr int kFMIR = PSCL_LANE_FRAME_MIRROR;

template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}

// rank counts of this lane's two children against the two children of lane pi(this lane):
// rg += [og < kg] + [ob < kg], rb += [og < kb] + [ob < kb], the other lane's keys read through the
// DPP permutation CTRL of og / ob (hand-scheduled: inline asm is not hazard-checked, so the first
// instruction waits out a VALU write of the key registers)
template <int CTRL>
__device__ __forceinline__ void rank_pair(uint32_t og, uint32_t ob, uint32_t kg, uint32_t kb, uint32_t& rg, uint32_t& rb) {
    uint32_t t;
    asm volatile(
        "s_nop 1\n\t"
        "v_sub_co_u32_dpp %0, vcc, %3, %5 quad_perm:[%7,%8,%9,%10] row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32 %1, vcc, 0, %1, vcc\n\t"
        "v_sub_co_u32_dpp %0, vcc, %4, %5 quad_perm:[%7,%8,%9,%10] row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32 %1, vcc, 0, %1, vcc\n\t"
        "v_sub_co_u32_dpp %0, vcc, %3, %6 quad_perm:[%7,%8,%9,%10] row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32 %2, vcc, 0, %2, vcc\n\t"
        "v_sub_co_u32_dpp %0, vcc, %4, %6 quad_perm:[%7,%8,%9,%10] row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32 %2, vcc, 0, %2, vcc"
        : "=&v"(t), "+v"(rg), "+v"(rb)
        : "v"(og), "v"(ob), "v"(kg), "v"(kb), "i"(CTRL & 3), "i"((CTRL >> 2) & 3), "i"((CTRL >> 4) & 3),
          "i"((CTRL >> 6) & 3)
        : "vcc");
}

// rank counts for the survivor selection (select_survivors): rg += [og < kg] + [ob < kg] (this
// lane's better child against the other lane's two children), rbb += [ob < kb] (its worse child
// against the other lane's worse child), the other lane read through the DPP permutation CTRL
template <int CTRL>
__device__ __forceinline__ void rank3(uint32_t og, uint32_t ob, uint32_t kg, uint32_t kb, uint32_t& rg, uint32_t& rbb) {
    uint32_t t;
    asm volatile(
        "s_nop 1\n\t"
        "v_sub_co_u32_dpp %0, vcc, %3, %5 quad_perm:[%7,%8,%9,%10] row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32 %1, vcc, 0, %1, vcc\n\t"
        "v_sub_co_u32_dpp %0, vcc, %4, %5 quad_perm:[%7,%8,%9,%10] row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32 %1, vcc, 0, %1, vcc\n\t"
        "v_sub_co_u32_dpp %0, vcc, %4, %6 quad_perm:[%7,%8,%9,%10] row_mask:0xf bank_mask:0xf\n\t"
        "v_addc_co_u32 %2, vcc, 0, %2, vcc"
        : "=&v"(t), "+v"(rg), "+v"(rbb)
        : "v"(og), "v"(ob), "v"(kg), "v"(kb), "i"(CTRL & 3), "i"((CTRL >> 2) & 3), "i"((CTRL >> 4) & 3),
          "i"((CTRL >> 6) & 3)
        : "vcc");
}

// lane i <-> 15 - i within a row: maps one 8-lane half of a 16-lane frame (G = 16, a whole row)
// onto the other
constexpr int kRMIR = 0x140;

// max / min / sum of v over the G lanes of each frame (G = 4: two quad_perm steps; G = 8: and
// the half-row mirror; G = 16: and the row mirror)
// the other row of a 32-lane frame (G = 32: two rows; DPP does not cross rows)
__device__ __forceinline__ uint32_t xrow32(uint32_t v) { return (uint32_t)__shfl_xor((int)v, 16); }

template <int G>
__device__ __forceinline__ uint32_t frame_max(uint32_t v) {
    uint32_t o = dpp32<kQX1>(v);
    v = o > v ? o : v;
    o = dpp32<kQX2>(v);
    v = o > v ? o : v;
    if constexpr (G >= 8) {
        o = dpp32<G >= 16 ? kHMIR : kFMIR>(v);
        v = o > v ? o : v;
    }
    if constexpr (G >= 16) {
        o = dpp32<kRMIR>(v);
        v = o > v ? o : v;
    }
    if constexpr (G == 32) {
        o = xrow32(v);
        v = o > v ? o : v;
    }
    return v;
}
template <int G>
__device__ __forceinline__ uint32_t frame_min(uint32_t v) {
    uint32_t o = dpp32<kQX1>(v);
    v = o < v ? o : v;
    o = dpp32<kQX2>(v);
    v = o < v ? o : v;
    if constexpr (G >= 8) {
        o = dpp32<G >= 16 ? kHMIR : kFMIR>(v);
        v = o < v ? o : v;
    }
    if constexpr (G >= 16) {
        o = dpp32<kRMIR>(v);
        v = o < v ? o : v;
    }
    if constexpr (G == 32) {
        o = xrow32(v);
        v = o < v ? o : v;
    }
    return v;
}
template <int G>
__device__ __forceinline__ uint32_t frame_sum(uint32_t v) {
    v += dpp32<kQX1>(v);
    v += dpp32<kQX2>(v);
    if constexpr (G >= 8) v += dpp32<G >= 16 ? kHMIR : kFMIR>(v);
    if constexpr (G >= 16) v += dpp32<kRMIR>(v);
    if constexpr (G == 32) v += xrow32(v);
    return v;
}

// Survivor selection of a full list (the L smallest of each frame's 2L children): this lane's
// better child key kg and worse child key kb (kb >= kg: the worse child pays |llr| more).  Keys are
// counted strictly below, so with distinct keys keep_g / win_b are exact; equal keys can give a
// wrong count, which the caller's certificate (exactly L survivors, margin between the largest
// survivor and the smallest non-survivor) always rejects.
//   PSCL_LANE_RANK3 = 1: rg = #{children below kg} (2L - 2 compares), d = the frame's number of
//     dropped better children, and a worse child survives iff it is among the d smallest worse
//     children (L - 1 compares): 3 compares per lane permutation.
//   0: both children ranked among all 2L (4 compares per permutation).
#ifndef PSCL_LANE_RANK3
#define PSCL_LANE_RANK3 1
#endif
template <int G, int LMAX>
__device__ __forceinline__ void select_survivors(uint32_t kg, uint32_t kb, bool& keep_g, bool& win_b) {
#if PSCL_LANE_RANK3
    uint32_t rg = 0, rbb = 0;
    rank3<kQX1>(kg, kb, kg, kb, rg, rbb);
    rank3<kQX2>(kg, kb, kg, kb, rg, rbb);
    rank3<kQX3>(kg, kb, kg, kb, rg, rbb);
    if constexpr (G >= 8) {  // the other quad of the frame's 8-lane half, through the half-row mirror
        const uint32_t mkg = dpp32<G >= 16 ? kHMIR : kFMIR>(kg), mkb = dpp32<G >= 16 ? kHMIR : kFMIR>(kb);
        rank3<kQID>(mkg, mkb, kg, kb, rg, rbb);
        rank3<kQX1>(mkg, mkb, kg, kb, rg, rbb);
        rank3<kQX2>(mkg, mkb, kg, kb, rg, rbb);
        rank3<kQX3>(mkg, mkb, kg, kb, rg, rbb);
    }
    // the row's other half (G >= 16): the row mirror (lane 15 - i) and the row mirror of the half-row
    // mirror (lane i + 8 or i - 8), each with the quad permutations; G = 32: then the other row's 16
    // lanes, brought over by a bpermute (xor 16), the same way
    auto quads16 = [&](uint32_t ok, uint32_t ob) {
        rank3<kQID>(ok, ob, kg, kb, rg, rbb);
        rank3<kQX1>(ok, ob, kg, kb, rg, rbb);
        rank3<kQX2>(ok, ob, kg, kb, rg, rbb);
        rank3<kQX3>(ok, ob, kg, kb, rg, rbb);
    };
    if constexpr (G >= 16) {
        quads16(dpp32<kRMIR>(kg), dpp32<kRMIR>(kb));
        quads16(dpp32<kRMIR>(dpp32<kHMIR>(kg)), dpp32<kRMIR>(dpp32<kHMIR>(kb)));
    }
    if constexpr (G == 32) {
        const uint32_t xg = xrow32(kg), xb = xrow32(kb);
        quads16(xg, xb);
        quads16(dpp32<kHMIR>(xg), dpp32<kHMIR>(xb));
        quads16(dpp32<kRMIR>(xg), dpp32<kRMIR>(xb));
        quads16(dpp32<kRMIR>(dpp32<kHMIR>(xg)), dpp32<kRMIR>(dpp32<kHMIR>(xb)));
    }
    keep_g = rg < (uint32_t)LMAX;
    const uint32_t d = frame_sum<G>(keep_g ? 0u : 1u);
    win_b = rbb < d;
#else
    static_assert(G <= 8, "the two-rank selection is built for frames of at most 8 lanes");
    uint32_t rg = 0, rb = kg < kb ? 1u : 0u;
    rank_pair<kQX1>(kg, kb, kg, kb, rg, rb);
    rank_pair<kQX2>(kg, kb, kg, kb, rg, rb);
    rank_pair<kQX3>(kg, kb, kg, kb, rg, rb);
    if constexpr (G == 8) {
        const uint32_t mkg = dpp32<kFMIR>(kg), mkb = dpp32<kFMIR>(kb);
        rank_pair<kQID>(mkg, mkb, kg, kb, rg, rb);
        rank_pair<kQX1>(mkg, mkb, kg, kb, rg, rb);
        rank_pair<kQX2>(mkg, mkb, kg, kb, rg, rb);
        rank_pair<kQX3>(mkg, mkb, kg, kb, rg, rb);
    }
    keep_g = rg < (uint32_t)LMAX;
    win_b = rb < (uint32_t)LMAX;
#endif
}

// position of the j-th set bit (j < popcount(m)) of a mask of at most 32 bits, branch-free
__device__ __forceinline__ uint32_t nth_set_bit16(uint32_t m, uint32_t j);
__device__ __forceinline__ uint32_t nth_set_bit32(uint32_t m, uint32_t j) {
    const uint32_t c16 = __builtin_popcount(m & 0xffffu);
    const bool h16 = j >= c16;
    return (h16 ? 16u : 0u) + nth_set_bit16(h16 ? (m >> 16) : (m & 0xffffu), h16 ? j - c16 : j);
}

// position of the j-th set bit (j < popcount(m)) of a mask of at most 16 bits, branch-free
__device__ __forceinline__ uint32_t nth_set_bit16(uint32_t m, uint32_t j) {
    const uint32_t c8 = __builtin_popcount(m & 255u);
    const bool h8 = j >= c8;
    j = h8 ? j - c8 : j;
    m = h8 ? (m >> 8) : (m & 255u);
    const uint32_t c4 = __builtin_popcount(m & 15u);
    const bool h4 = j >= c4;
    j = h4 ? j - c4 : j;
    m = h4 ? (m >> 4) : (m & 15u);
    const uint32_t c2 = __builtin_popcount(m & 3u);
    const bool h2 = j >= c2;
    j = h2 ? j - c2 : j;
    m = h2 ? (m >> 2) : m;
    const bool h1 = j >= (m & 1u);
    return (h8 ? 8u : 0u) + (h4 ? 4u : 0u) + (h2 ? 2u : 0u) + (h1 ? 1u : 0u);
}

// position of the j-th set bit (j < popcount(m)) of a mask of at most 8 bits, branch-free
__device__ __forceinline__ uint32_t nth_set_bit8(uint32_t m, uint32_t j) {
    const uint32_t c4 = __builtin_popcount(m & 15u);
    const bool h4 = j >= c4;
    j = h4 ? j - c4 : j;
    m = h4 ? (m >> 4) : (m & 15u);
    const uint32_t c2 = __builtin_popcount(m & 3u);
    const bool h2 = j >= c2;
    j = h2 ? j - c2 : j;
    m = h2 ? (m >> 2) : m;
    const bool h1 = j >= (m & 1u);
    return (h4 ? 4u : 0u) + (h2 ? 2u : 0u) + (h1 ? 1u : 0u);
}

}  // namespace

#endif
