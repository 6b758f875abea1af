// scl_lane_long.hip -- the lane-per-path screening decoder for the longer codes (N = 256, 512,
// 1024; L = 4, 8; any information set) and its launch.
//
// The long-code form of scl128_lane.hip: a plain decode whose path
// metrics carry the bounded-error tail (pscl_softplus_tail_abs), every ordering decision
// certified by the absolute margin of an N-phase metric (2 N DELTA), a frame with an uncertain
// decision appended to P.amb_list and re-decoded exactly by scl_long_kernel (capi.cpp).  Results
// are therefore bit-identical to decode_scl (dl_scl_polar/polar/scl.py:108-209; any power-of-two
// N, scl.py:25-30).
//
// Mapping: one lane per list path, G = L lanes per frame, 64 / L frames per wavefront, the
// state of a frame in registers and LDS -- no global scratch (scl_long_kernel keeps one frame per
// wavefront and its trees in global memory, latency-bound at ~6 us per phase).
//   * phases run in blocks of 16 (a runtime loop over N / 16 blocks; the 16 positions of a block
//     unrolled): the information set is a runtime bitmask (one 16-bit slice per block, scalar);
//   * depths R = n-4 .. n-1 (node widths 16, 8, 4, 2) in LDS slots with lazy copies, as N = 128;
//   * depths 1..R recomputed from the channel row at every block start: element e < 16 of the
//     depth-R node of path q reduces the 2^R channel LLRs chan[e + 16 m] through R f/g levels,
//     level l a g node when bit (R - l) of the block index is set, with the left sibling's
//     partial sums (published per path in LDS by the path's lane).  The depth-1 f node is
//     path-independent and computed once per element.  N = 256 at L = 8 keeps the lane's 32
//     channel LLRs in registers; otherwise they are re-read (L2) at each block start;
//   * decided bits: the current block's 16 in a register (compile-time shifts within the block),
//     merged into N / 64 words at the block end; a clone pulls the words in use;
//   * list steps (frozen / growing / keep-better / one swap / ranked), the final order and the
//     epilogue as scl128_lane.hip, with the information-bit gather from N / 8 byte tables.
#include "scl_lane.h"

namespace {

template <int NL, int LMAX>
struct LongLaneLayout {
    static constexpr int N = 1 << NL;
    static constexpr int R = NL - 4;           // the widest stored depth (node width 16)
    static constexpr int G = LMAX;
    static constexpr int F = 64 / G;
    static constexpr int LOG_G = __builtin_ctz(G);
    static constexpr int OFF0 = 0;              // depth R:   [8][L][2] doubles
    static constexpr int OFF1 = 16 * LMAX;      // depth R+1: [4][L][2]
    static constexpr int OFF2 = 24 * LMAX;      // depth R+2: [2][L][2]
    static constexpr int OFF3 = 28 * LMAX;      // depth R+3: [1][L][2]
    // partial sums of the depth-1..R left siblings, per path: level l (node width N >> l) at
    // 32-bit word xoff(l) = sum of (N >> l') / 32 over l' < l, max(1, (N >> l) / 32) words
    template <int l>
    static constexpr int xoff = (N >> 5) - (N >> (4 + l));
    static constexpr int XWORDS = N / 32;
    static constexpr int OFFX = 30 * LMAX;      // [L][XWORDS] uint32
    static constexpr int RAW = OFFX + LMAX * XWORDS / 2;
    // frames start alternately on the two 128-byte halves of the 256-byte bank row (as N = 128)
    static constexpr int FSTRIDE = RAW + (((16 - RAW) % 32) + 32) % 32;
};

#ifndef PSCL_LANE_LONG_WAVES_PER_EU
#define PSCL_LANE_LONG_WAVES_PER_EU 2
#endif
// N = 1024 (and N = 512 at L = 16, 32): the element recompute holds 64 channel LLRs (128 VGPRs); at
// 2 waves/SIMD (256 VGPRs) it spills (592 bytes of scratch per lane at N = 1024, 120-168 at N = 512,
// L >= 16), at 1 (512) none -- LDS allows 6 wavefronts per CU either way.  Measured (tools/long_bench.py, profiles/r05j_long_*): 3.42 M frames/s at 1 against
// 2.60 M at 2 (4.36 M against 3.02 M pipelined)
#ifndef PSCL_LANE_LONG1024_WAVES_PER_EU
#define PSCL_LANE_LONG1024_WAVES_PER_EU 1
#endif

// word k of the register array u, k wave-uniform.  The selects are inline asm (v_cndmask with the
// wave-uniform condition in an SGPR pair): left as C, the compiler turned the select chain into a
// load from a private copy of u indexed by k, i.e. u kept in scratch and stored on every pull
// (48 / 80 / 144 B of scratch per lane at N = 256 / 512 / 1024)
template <int NW>
__device__ __forceinline__ uint64_t uword(const uint64_t (&u)[NW], int k) {
    uint32_t lo = (uint32_t)u[0], hi = (uint32_t)(u[0] >> 32);
    const int ku = __builtin_amdgcn_readfirstlane(k);  // (uniform: the condition lives in SGPRs)
#pragma unroll
    for (int i = 1; i < NW; ++i) {
        const uint32_t c = __builtin_amdgcn_readfirstlane(ku == i ? 0xffffffffu : 0u);
        const uint64_t m = ((uint64_t)c << 32) | c;
        asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(lo) : "v"(lo), "v"((uint32_t)u[i]), "s"(m));
        asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(hi) : "v"(hi), "v"((uint32_t)(u[i] >> 32)), "s"(m));
    }
    return ((uint64_t)hi << 32) | lo;
}

// the bits of NV g nodes of element e (node m: bit e + 16 (m & 1) of word wb[m >> 1]) moved to bit 31
// of o[m]: one 64-bit shift of a word pair serves two nodes (bit e of words 2k and 2k + 1, or bit
// e + 16), for g_node_bit31 -- half the shifts of g_node_wbit
template <int NV>
__device__ __forceinline__ void bits31(const uint32_t* wb, uint32_t e, uint32_t (&o)[NV]) {
    if constexpr (NV >= 4) {
#pragma unroll
        for (int k = 0; k < NV / 4; ++k) {
            const uint64_t pr = ((uint64_t)wb[2 * k + 1] << 32) | wb[2 * k];
            const uint64_t a = pr << (31u - e), c = pr << (15u - e);
            o[4 * k] = (uint32_t)a;
            o[4 * k + 1] = (uint32_t)c;
            o[4 * k + 2] = (uint32_t)(a >> 32);
            o[4 * k + 3] = (uint32_t)(c >> 32);
        }
    } else {
#pragma unroll
        for (int m = 0; m < NV; ++m) o[m] = wb[m >> 1] << (31u - e - 16u * (m & 1));
    }
}

template <int NL, int LMAX>
__global__ void __launch_bounds__(64, (NL == 10 || (NL == 9 && LMAX >= 16)) ? PSCL_LANE_LONG1024_WAVES_PER_EU
                                                                           : PSCL_LANE_LONG_WAVES_PER_EU)
    scl_lane_long_kernel(const pscl_decode_params P) {
    static_assert(LMAX == 4 || LMAX == 8 || LMAX == 16 || LMAX == 32,
                  "the lane-per-path decoder is built for L = 4, 8, 16 and 32");
    static_assert(NL >= 7 && NL <= 10, "N = 128 .. 1024");
    using Ly = LongLaneLayout<NL, LMAX>;
    constexpr int N = Ly::N, R = Ly::R, G = Ly::G, F = Ly::F, LOG_G = Ly::LOG_G;
    constexpr int CE = 1 << R;          // channel LLRs per depth-R element
    constexpr int NW = N / 64;          // decided-bit words per path
    // depth-R elements per lane at a block start; G = 32: the lanes p and p + 16 share element p % 16,
    // each recomputing it for half of the paths (those of parity p / 16)
    constexpr int EPL = G == 32 ? 1 : 16 / G;
    constexpr uint32_t GM = G == 32 ? 0xffffffffu : (1u << G) - 1u;
    // slot-table fields: 4 bits per stored depth (L <= 16) or 5 (L = 32)
    constexpr int SB = LMAX > 16 ? 5 : 4;
    constexpr uint32_t SFULL = (1u << (4 * SB)) - 1u, SREP = SB == 4 ? 0x1111u : 0x8421u;
    constexpr bool CREG = EPL * CE <= 32;  // N = 256, L = 8: the lane's channel LLRs stay in registers
    // every metric carries N tail terms: two metrics differ from their exact values by < 2 N DELTA.
    // Metrics in bits (PSCL_LANE_BITS, scl128_lane.hip): the channel LLRs scaled by log2 e as they
    // are loaded, the tail without its multiplies, DELTA = PSCL_TAIL2_DELTA (glibc_softplus.h: its
    // tree term covers n <= 10 levels, (2 n + 2) u S' < 2^-31 for S' < 2^17)
    constexpr bool BITS = PSCL_LANE_BITS;
    constexpr double MARGIN = 2.0 * N * (BITS ? PSCL_TAIL2_DELTA : PSCL_TAIL_ABS_DELTA) * 1.0001;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* const A = reinterpret_cast<double*>(smem);
    const int lane = threadIdx.x & 63;
    const int fl = lane >> LOG_G, p = lane & (G - 1), gbase = lane & ~(G - 1);
    const int pe = G == 32 ? (p & 15) : p;  // the lane's first depth-R element (EPL above)
    double* const Af = A + fl * Ly::FSTRIDE;
    uint32_t* const XS = reinterpret_cast<uint32_t*>(Af + Ly::OFFX);
    const uint8_t* const GT = reinterpret_cast<const uint8_t*>(P.epi_table);        // [N/8][256] u-byte -> info bits
    const uint32_t* const ST = reinterpret_cast<const uint32_t*>(GT + (N / 8) * 256);  // [K/4][16] nibble -> syndrome
    const int K = P.K, W = P.W;
    auto hiw = [](double m) { return (uint32_t)(pscl_asu64(m) >> 32); };
    // the margin-raised key as one VOP3 fma with the factor in an SGPR (scl128_lane.hip)
    auto hiw_up = [&](double m) {
        double r;
        asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(m), "s"(1.0 + 0x1p-40), "v"(MARGIN));
        return hiw(r);
    };
    auto frame_bits = [&](uint64_t m) { return (uint32_t)(m >> gbase) & GM; };
    auto slot_rel = [](uint32_t tab, int dr) { return (int)((tab >> (SB * dr)) & ((1u << SB) - 1u)); };

    int cfe = 0, cbe = 0, cpe = 0, cpb = 0;  // this lane's error counts (flushed at the end)
    for (int64_t f0 = (int64_t)blockIdx.x * F; f0 < P.B; f0 += (int64_t)gridDim.x * F) {
        const int64_t fi = f0 + fl;
        const bool fvalid = fi < P.B;
        const int64_t frow = fvalid ? fi : f0;  // (a tail wave's empty slots decode a copy of frame f0)
        const double* chan = P.llr + frow * N;
        // the lane's depth-R elements e_h = p + G h (h < EPL) reduce ch[m] = chan[e_h + 16 m]
        double c[CREG ? EPL * CE : 1];
        uint64_t amb;
        {
            double cs = 0.0;  // NaN / overflow guard over the lane's channel LLRs (the 8 lanes: all N)
#pragma unroll
            for (int h = 0; h < EPL; ++h)
#pragma unroll
                for (int m = 0; m < CE; ++m) {
                    const double v = BITS ? chan[pe + G * h + 16 * m] * PSCL_LOG2E_F64 : chan[pe + G * h + 16 * m];
                    if constexpr (CREG) c[CE * h + m] = v;
                    cs = cs + fabs(v);
                }
            amb = wmask(!(cs < (BITS ? PSCL_TAIL2_CHAN_SUM_G(G) : 0x1p25)));
        }
        const uint64_t vmask = wmask(fvalid);

        double metric = 0.0;
        uint64_t u[NW];
#pragma unroll
        for (int k = 0; k < NW; ++k) u[k] = 0;
        uint32_t ub = 0;       // bits of the current block's phases
        uint32_t tab = 0;      // LDS slot of depths R..R+3 (4 bits each)
        uint32_t lastbit = 0;  // the bit decided at the previous phase
        int cnt = 1;           // live paths (wave-uniform)

        // pull the state of lane src (words of phases below block b only)
        auto pull_u = [&](int src, int b) {
#pragma unroll
            for (int k = 0; k < NW; ++k)
                if (64 * k < 16 * b) u[k] = shfl_u64(u[k], src);
        };

        for (int b = 0; b < N / 16; ++b) {
            const uint32_t info16 = (uint32_t)(P.info_words[b >> 2] >> (16 * (b & 3))) & 0xffffu;

            // ---- depths 1..R from the channel (block start)
            {
                // left-sibling partial sums of every g level, published by each path's lane
                if (b) {
                    static_for<R>([&](auto LI) {
                        constexpr int l = 1 + decltype(LI)::value;
                        constexpr int w = N >> l;  // node width at depth l
                        const int k = b >> (R - l);
                        if (k & 1) {
                            const int lo = (k - 1) * w;  // left sibling u[lo, lo + w)
                            uint32_t* xo = XS + p * Ly::XWORDS + Ly::template xoff<l>;
                            if constexpr (w >= 64) {
                                constexpr int nw = w / 64;
                                uint64_t x[nw];
#pragma unroll
                                for (int i = 0; i < nw; ++i) x[i] = polar_transform64(uword<NW>(u, (lo >> 6) + i));
#pragma unroll
                                for (int s = 1; s < nw; s <<= 1)
#pragma unroll
                                    for (int i = 0; i < nw; ++i)
                                        if (!(i & s)) x[i] ^= x[i + s];
#pragma unroll
                                for (int i = 0; i < nw; ++i) {
                                    xo[2 * i] = (uint32_t)x[i];
                                    xo[2 * i + 1] = (uint32_t)(x[i] >> 32);
                                }
                            } else {
                                const uint32_t seg = (uint32_t)(uword<NW>(u, lo >> 6) >> (lo & 63));
                                xo[0] = w == 32 ? polar_transform32(seg) : polar_transform16(seg & 0xffffu);
                            }
                        }
                    });
                    wave_lds_fence();
                }
                const bool r1 = (b >> (R - 1)) & 1;
                const bool r2 = (b >> (R - 2)) & 1;
                auto elem = [&](auto HC) {
                    const int h = HC;
                    const uint32_t e = (uint32_t)(pe + G * h);
                    // every path of the element: depths 1-2 by first(q, xq, v), then depths 3..R
                    auto paths = [&](auto&& first) {
                        auto path = [&](int q0) {
                            // lane p takes path (q0 + p) mod L: the lanes' stores hit distinct bank groups
                            // (G = 32: q0 of the lane's parity, rotated by 2 (p % 16), keeping it)
                            const int q = cnt == LMAX ? ((q0 + (G == 32 ? 2 * (p & 15) : p)) & (LMAX - 1)) : q0;
                            const uint32_t* xq = XS + q * Ly::XWORDS;
                            double v[CE / 4];  // depth-2 values at e + 16 m
                            first(xq, v);
                            static_for<R - 2>([&](auto LI) {
                                constexpr int l = 3 + decltype(LI)::value;
                                constexpr int nl = CE >> l;  // values per element at depth l
                                if ((b >> (R - l)) & 1) {
                                    uint32_t o[nl];
                                    bits31<nl>(xq + Ly::template xoff<l>, e, o);
#pragma unroll
                                    for (int m = 0; m < nl; ++m) v[m] = g_node_bit31(v[m], v[m + nl], o[m]);
                                } else {
#pragma unroll
                                    for (int m = 0; m < nl; ++m) v[m] = f_minsum(v[m], v[m + nl]);
                                }
                            });
                            // element e of slot q: pair index e & 7, half e >> 3 ([8][L][2] layout)
                            Af[Ly::OFF0 + ((e & 7) * LMAX + q) * 2 + (e >> 3)] = v[0];
                        };
                        if constexpr (G == 32) {  // the paths of parity p / 16
#pragma unroll
                            for (int i = 0; i < LMAX / 2; ++i)
                                if (2 * i + (p >> 4) < cnt) path(2 * i + (p >> 4));
                        } else if constexpr (CREG) {
#pragma unroll
                            for (int q0 = 0; q0 < LMAX; ++q0)
                                if (q0 < cnt) path(q0);
                        } else {
#pragma nounroll
                            for (int q0 = 0; q0 < cnt; ++q0) path(q0);
                        }
                    };
                    double ch[CE];
                    if constexpr (CREG) {
#pragma unroll
                        for (int m = 0; m < CE; ++m) ch[m] = c[CE * h + m];
                    } else {
#pragma unroll
                        for (int m = 0; m < CE; ++m) ch[m] = BITS ? chan[e + 16 * m] * PSCL_LOG2E_F64 : chan[e + 16 * m];
                    }
                    if (!r1) {
                        // depth 1 before phase N/2: the same f node for every path (the channel
                        // values die here: only the shared half-size set stays live)
                        double v1s[CE / 2];
#pragma unroll
                        for (int m = 0; m < CE / 2; ++m) v1s[m] = f_minsum(ch[m], ch[m + CE / 2]);
                        if (r2)
                            paths([&](const uint32_t* xq, double* v) {
                                uint32_t o[CE / 4];
                                bits31<CE / 4>(xq + Ly::template xoff<2>, e, o);
#pragma unroll
                                for (int m = 0; m < CE / 4; ++m) v[m] = g_node_bit31(v1s[m], v1s[m + CE / 4], o[m]);
                            });
                        else
                            paths([&](const uint32_t* xq, double* v) {
#pragma unroll
                                for (int m = 0; m < CE / 4; ++m) v[m] = f_minsum(v1s[m], v1s[m + CE / 4]);
                            });
                    } else {
                        // depths 1 and 2 together from the channel (depth-1 pair (m, m + CE/4))
                        auto d1 = [&](const uint32_t (&o1)[CE / 2], int m) { return g_node_bit31(ch[m], ch[m + CE / 2], o1[m]); };
                        if (r2)
                            paths([&](const uint32_t* xq, double* v) {
                                uint32_t o1[CE / 2], o2[CE / 4];
                                bits31<CE / 2>(xq + Ly::template xoff<1>, e, o1);
                                bits31<CE / 4>(xq + Ly::template xoff<2>, e, o2);
#pragma unroll
                                for (int m = 0; m < CE / 4; ++m) v[m] = g_node_bit31(d1(o1, m), d1(o1, m + CE / 4), o2[m]);
                            });
                        else
                            paths([&](const uint32_t* xq, double* v) {
                                uint32_t o1[CE / 2];
                                bits31<CE / 2>(xq + Ly::template xoff<1>, e, o1);
#pragma unroll
                                for (int m = 0; m < CE / 4; ++m) v[m] = f_minsum(d1(o1, m), d1(o1, m + CE / 4));
                            });
                    }
                };
                if constexpr (CREG) {
                    static_for<EPL>([&](auto HC) { elem(HC); });
                } else {
                    // one element at a time: its 2^R channel LLRs are the recompute's largest live set
#pragma nounroll
                    for (int h = 0; h < EPL; ++h) elem(h);
                }
                wave_lds_fence();
            }

            auto phase = [&](auto TC) {
                constexpr int t = decltype(TC)::value;
                constexpr int start = t ? NL - __builtin_ctz((unsigned)t) : R;  // (t = 0: depth R just written)
                const bool is_info = (info16 >> t) & 1u;
                // ---- depths R+1 .. n-1: this lane's own path; the first rewritten depth reads the parent slot
                if constexpr (start <= NL - 1) {
                    uint32_t xsb = 0;  // partial sums of the first rewritten node's left sibling (g node)
                    if constexpr (t) {
                        constexpr int w = 1 << (NL - start);
                        xsb = polar_transform8((ub >> (t - w)) & ((1u << w) - 1u));
                    }
                    static_for<3>([&](auto DI) {
                        constexpr int dr = 1 + decltype(DI)::value;  // depth R + dr
                        constexpr int D = R + dr;
                        if constexpr (D >= start) {
                            constexpr int Wd = 1 << (NL - D), HW = Wd / 2;
                            constexpr int OFF_IN = dr == 1 ? Ly::OFF0 : (dr == 2 ? Ly::OFF1 : Ly::OFF2);
                            constexpr int OFF_OUT = dr == 1 ? Ly::OFF1 : (dr == 2 ? Ly::OFF2 : Ly::OFF3);
                            constexpr bool first = D == start || (dr == 1 && t == 0);
                            constexpr bool is_g = D == start && t != 0;
                            const int sin = (t == 0 && dr == 1) ? p : (first ? slot_rel(tab, dr - 1) : p);
                            const double* in = Af + OFF_IN + sin * 2;
                            double o[Wd];
#pragma unroll
                            for (int k = 0; k < Wd; ++k) {
                                const double2 ab = *reinterpret_cast<const double2*>(in + k * LMAX * 2);
                                o[k] = is_g ? g_node(ab.x, ab.y, (xsb >> k) & 1u) : f_minsum(ab.x, ab.y);
                            }
                            double* out = Af + OFF_OUT + p * 2;
#pragma unroll
                            for (int k = 0; k < HW; ++k)
                                *reinterpret_cast<double2*>(out + k * LMAX * 2) = make_double2(o[k], o[k + HW]);
                            wave_lds_fence();
                        }
                    });
                    // this path's own slot at every depth rewritten this phase
                    constexpr int s0 = start - R;
                    constexpr uint32_t mask = (SFULL << (SB * s0)) & SFULL;
                    tab = (tab & ~mask) | ((uint32_t)p * SREP & mask);
                }
                // ---- leaf LLR and metric tail (scl.py:80-82, 102-105)
                const double2 lab = *reinterpret_cast<const double2*>(Af + Ly::OFF3 + (start <= NL - 1 ? p : slot_rel(tab, 3)) * 2);
                const double lam = (t & 1) ? g_node(lab.x, lab.y, lastbit) : f_minsum(lab.x, lab.y);
                const double Lt = BITS ? pscl_softplus_tail2(lam) : pscl_softplus_tail_abs(lam);
                if (!is_info) {  // frozen: bit 0 (scl.py:149-153)
                    metric = metric + (relu_neg(lam) + Lt);
                    lastbit = 0;
                    return;
                }
                // information phase: better child (along the LLR sign) mg, worse child mb
                const double mg = metric + Lt, mb = mg + fabs(lam);
                const uint32_t gbit = sign_bit(lam);
                if (cnt < LMAX) {
                    // growing list: every child survives; bit-1 children to lanes cnt..2cnt-1
                    const double m0 = gbit ? mb : mg, m1 = gbit ? mg : mb;
                    const int src = gbase + (p & (cnt - 1));
                    const uint32_t bt = (p & cnt) ? 1u : 0u;
                    const uint64_t pm1 = shfl_u64(pscl_asu64(m1), src);
                    metric = bt ? pscl_asf64(pm1) : m0;  // (lanes below cnt: src is the lane itself)
                    pull_u(src, b);
                    ub = bperm32(ub, src) | (bt << t);
                    tab = bperm32(tab, src);
                    lastbit = bt;
                    cnt *= 2;
                    return;
                }
                // full list: keep the better children when every worse child clears the largest
                // better child by the margin (the stable sort's outcome; ties never reach the sort)
                const uint32_t kgu = hiw_up(mg), kb = hiw(mb);
                const uint32_t mx = frame_max<G>(kgu);
                const bool bad = kb <= mx;
                const uint64_t badm = wmask(bad);
                metric = mg;
                uint32_t bt = gbit;
                if ((badm & vmask) != 0) {
                    const uint32_t bad8 = frame_bits(badm);
                    int src;
                    bool take;  // this lane's path becomes a pulled worse child
#if PSCL_LANE_SWAP
                    if ((wmask(__builtin_popcount(bad8) > 1) & vmask) == 0) {
                        // one swap per frame at most (scl128_lane.hip): the largest better child gives
                        // way to the one unclear worse child, certified by the margin or deferred
                        const uint32_t kg = hiw(mg);
                        const uint32_t gmaxh = frame_max<G>(kg);
                        const bool ismax = kg == gmaxh;
                        const uint32_t nmax = frame_sum<G>(ismax ? 1u : 0u);
                        const uint32_t g2u = frame_max<G>(ismax ? 0u : kgu);
                        const uint32_t wu = frame_max<G>(bad ? hiw_up(mb) : 0u);
                        const bool swap = bad8 != 0;
                        amb |= wmask(swap && !(nmax == 1u && g2u < gmaxh && wu < gmaxh)) & vmask;
                        src = (gbase + (int)__builtin_ctzll((uint64_t)bad8 | (1ull << G))) & 63;
                        take = swap && ismax;
                    } else
#endif
                    {
                        // rank the 2L children of each frame (select_survivors) and certify
                        const uint32_t kg = hiw(mg);
                        bool keep_g, win_b;
                        select_survivors<G, LMAX>(kg, kb, keep_g, win_b);
                        const uint32_t kbu = hiw_up(mb);
                        const uint32_t su = keep_g ? (win_b ? kbu : kgu) : (win_b ? kbu : 0u);
                        const uint32_t nm = keep_g ? (win_b ? 0xffffffffu : kb) : kg;
                        const uint32_t nsurv = frame_sum<G>((keep_g ? 1u : 0u) + (win_b ? 1u : 0u));
                        const uint32_t smax = frame_max<G>(su), nmin = frame_min<G>(nm);
                        amb |= wmask(!(nsurv == (uint32_t)LMAX && nmin > smax)) & vmask;
                        const uint32_t f8 = frame_bits(wmask(!keep_g)), w8 = frame_bits(wmask(win_b));
                        const uint32_t j = __builtin_popcount(f8 & ((1u << p) - 1u));
                        src = gbase + (int)(G == 32 ? nth_set_bit32(w8, j) : G == 16 ? nth_set_bit16(w8, j) : nth_set_bit8(w8, j));
                        take = !keep_g;
                    }
                    // the worse child's bit rides on the table word
                    const uint32_t tw = tab | ((gbit ^ 1u) << 31);
                    const uint64_t pmb = shfl_u64(pscl_asu64(mb), src);
                    const uint32_t ptw = bperm32(tw, src);
                    const uint32_t pub = bperm32(ub, src);
                    // (word by word: one pulled word live at a time)
#pragma unroll
                    for (int k = 0; k < NW; ++k)
                        if (64 * k < 16 * b) {
                            const uint64_t x = shfl_u64(u[k], src);
                            u[k] = take ? x : u[k];
                        }
                    if (take) {
                        metric = pscl_asf64(pmb);
                        ub = pub;
                        tab = ptw & 0x7fffffffu;
                        bt = ptw >> 31;
                    }
                }
                ub |= bt << t;
                lastbit = bt;
            };
            static_for<16>([&](auto TC) { phase(TC); });
            // the block's bits into their word (a uniform branch per word, the OR in asm: as plain
            // C the compiler made this a store into a private copy of u indexed by b / 4, which
            // kept u in scratch at N = 1024)
            {
                const int kb = __builtin_amdgcn_readfirstlane(b >> 2);
                const uint64_t add = (uint64_t)ub << (16 * (b & 3));
#pragma unroll
                for (int k = 0; k < NW; ++k)
                    if (k == kb) {
                        uint32_t lo = (uint32_t)u[k], hi = (uint32_t)(u[k] >> 32);
                        asm volatile("v_or_b32 %0, %0, %1" : "+v"(lo) : "v"((uint32_t)add));
                        asm volatile("v_or_b32 %0, %0, %1" : "+v"(hi) : "v"((uint32_t)(add >> 32)));
                        u[k] = ((uint64_t)hi << 32) | lo;
                    }
            }
            ub = 0;
        }

        // ---- epilogue: candidates u[info_set], CRC syndrome, final list order certified,
        // best = first CRC pass in list order (scl.py:176-209)
        uint64_t ib[NW];
#pragma unroll
        for (int k = 0; k < NW; ++k) ib[k] = 0;
        {
            int off = 0;  // information bits before byte k (wave-uniform)
            // words of u by a compile-time index (the byte loop inside may stay rolled: at N = 1024
            // a rolled loop over all N / 8 bytes indexed u by k / 8, which put u in scratch)
#pragma unroll
            for (int kw = 0; kw < NW; ++kw) {
                const uint64_t uw = u[kw], iw = P.info_words[kw];
                for (int j = 0; j < 8; ++j) {
                    const int k = 8 * kw + j;
                    const uint32_t byte = (uint32_t)((uw >> (8 * j)) & 255u);
                    const uint64_t cb = GT[k * 256 + byte];
                    const int wi = off >> 6, sb = off & 63;
#pragma unroll
                    for (int w = 0; w < NW; ++w) {
                        if (w == wi) ib[w] |= cb << sb;
                        if (w == wi + 1 && sb > 56) ib[w] |= cb >> (64 - sb);
                    }
                    off += __builtin_popcount((uint32_t)((iw >> (8 * j)) & 255u));
                }
            }
        }
        uint32_t syn = 0;
        if (P.has_crc) {
            const int k4 = (K + 3) >> 2;
#pragma unroll
            for (int w = 0; w < NW; ++w)
#pragma unroll
                for (int jn = 0; jn < 16; ++jn) {
                    const int m = 16 * w + jn;
                    if (m < k4) syn ^= ST[m * 16 + (uint32_t)((ib[w] >> (4 * jn)) & 15u)];
                }
        }
        // list position = rank of the metric among the frame's L (high words); certified when all
        // pairs are apart by the margin (then the ranks are distinct and equal the exact order)
        const uint32_t kh = hiw(metric), ku = hiw_up(metric);
        uint32_t r = 0;
        bool near = false;
        auto cmp_perm = [&](uint32_t oh, uint32_t ou) {
            r += oh < kh ? 1u : 0u;
            near = near || !(ku < oh || ou < kh);
        };
        cmp_perm(dpp32<kQX1>(kh), dpp32<kQX1>(ku));
        cmp_perm(dpp32<kQX2>(kh), dpp32<kQX2>(ku));
        cmp_perm(dpp32<kQX3>(kh), dpp32<kQX3>(ku));
        // the other quads of the frame: G = 8 the half-row mirror's; G = 16 also the row mirror's and
        // the row mirror of the half-row mirror's (select_survivors, scl_lane.h)
        auto cmp_quad = [&](uint32_t mh, uint32_t mu) {
            cmp_perm(mh, mu);
            cmp_perm(dpp32<kQX1>(mh), dpp32<kQX1>(mu));
            cmp_perm(dpp32<kQX2>(mh), dpp32<kQX2>(mu));
            cmp_perm(dpp32<kQX3>(mh), dpp32<kQX3>(mu));
        };
        if constexpr (G >= 8) cmp_quad(dpp32<kHMIR>(kh), dpp32<kHMIR>(ku));
        if constexpr (G >= 16) {
            cmp_quad(dpp32<kRMIR>(kh), dpp32<kRMIR>(ku));
            cmp_quad(dpp32<kRMIR>(dpp32<kHMIR>(kh)), dpp32<kRMIR>(dpp32<kHMIR>(ku)));
        }
        if constexpr (G == 32) {  // the frame's other row
            const uint32_t xh = xrow32(kh), xu = xrow32(ku);
            cmp_quad(xh, xu);
            cmp_quad(dpp32<kHMIR>(xh), dpp32<kHMIR>(xu));
            cmp_quad(dpp32<kRMIR>(xh), dpp32<kRMIR>(xu));
            cmp_quad(dpp32<kRMIR>(dpp32<kHMIR>(xh)), dpp32<kRMIR>(dpp32<kHMIR>(xu)));
        }
        amb |= wmask(near) & vmask;
        const bool famb = ((amb >> gbase) & (uint64_t)GM) != 0;
        if (famb && p == 0 && fvalid) P.amb_list[atomicAdd(P.amb_count, 1)] = fi;
        const uint32_t pass = P.has_crc ? (syn == 0 ? 1u : 0u) : 1u;
        const uint32_t keyb = pass ? r : (uint32_t)LMAX + r;
        const uint32_t kbest = frame_min<G>(keyb);
        if (fvalid && !famb && keyb == kbest) {
            const int best = (int)(kbest & (uint32_t)(LMAX - 1));
            const bool bpass = kbest < (uint32_t)LMAX;
            if (P.best)
#pragma unroll
                for (int w = 0; w < NW; ++w)
                    if (w < W) P.best[fi * W + w] = ib[w];
            if (P.flags) P.flags[fi] = (uint8_t)((bpass ? PSCL_FLAG_CRC_PASS : 0u) | (uint32_t)best);
            if (P.n_paths) P.n_paths[fi] = LMAX;
            if (P.ref) {  // run_fer_sweep.py:91-109, run_ber_sweep.py:77-82,156
                uint64_t rw[NW];
#pragma unroll
                for (int w = 0; w < NW; ++w) rw[w] = w < W ? P.ref[fi * W + w] : ib[w];
                tally_errors(ib, rw, NW, P.k_payload, bpass, cfe, cbe, cpe, cpb);
            }
        }
        wave_lds_fence();
    }
    if (P.ref) {
        flush_counts_p(P, blockIdx.x, cfe, cbe, cpe, cpb);
        if (blockIdx.x == 0 && threadIdx.x == 0)
            atomicAdd(reinterpret_cast<unsigned long long*>(P.counters) + PSCL_CNT_FRAMES, (unsigned long long)P.B);
    }
}

int64_t lane_long_grid(const pscl_decode_params& P) {
    const int F = 64 / P.L;
    const int64_t g0 = (P.B + F - 1) / F;
    const int64_t cap = P.ref && !P.cpart ? PSCL_LANE_COUNT_GRID : (1 << 20);
    return g0 < 1 ? 1 : (g0 > cap ? cap : g0);
}

template <int NL, int LMAX>
hipError_t launch_lane_long(const pscl_decode_params& P, hipStream_t s) {
    using Ly = LongLaneLayout<NL, LMAX>;
    const int64_t grid = lane_long_grid(P);
    hipLaunchKernelGGL((scl_lane_long_kernel<NL, LMAX>), dim3((unsigned)grid), dim3(64), Ly::F * Ly::FSTRIDE * 8, s, P);
    return hipGetLastError();
}

}  // namespace

#ifndef PSCL_LANE_LONG
#define PSCL_LANE_LONG 1
#endif

// the screening launch of this plain decode can run the runtime-information-set lane-per-path
// kernel: N = 256, 512 or 1024 (every long code), or N = 128 (the codes without a compiled-in
// screening kernel: pscl_launch_decode takes the compiled-in ones first); L = 4 or 8, plain
// channel rows, at least log2 L information bits (a full list)
int pscl_lane_long_available(const pscl_decode_params& P) {
    if (!PSCL_LANE_LONG || !P.apx || P.force || P.sc_hard || P.rm_E || P.fidx || P.d_count || P.elist) return 0;
    if (!P.info_words || !P.epi_table || P.out_by_row) return 0;
    if (P.L != 32 && P.L != 16 && P.L != 8 && P.L != 4) return 0;
    if (P.N != 128 && P.N != 256 && P.N != 512 && P.N != 1024) return 0;
    return P.K >= __builtin_ctz((unsigned)P.L);
}

int64_t pscl_lane_long_grid(const pscl_decode_params& P) { return lane_long_grid(P); }

hipError_t pscl_launch_lane_long(const pscl_decode_params& P, hipStream_t s) {
    if (!pscl_lane_long_available(P)) return hipErrorInvalidValue;
#define PSCL_LL(NL_)                                                                                        \
    (P.L == 32 ? launch_lane_long<NL_, 32>(P, s) : P.L == 16 ? launch_lane_long<NL_, 16>(P, s)                \
                                                 : P.L == 8 ? launch_lane_long<NL_, 8>(P, s) : launch_lane_long<NL_, 4>(P, s))
    switch (P.N) {
        case 128: return PSCL_LL(7);
        case 256: return PSCL_LL(8);
        case 512: return PSCL_LL(9);
        default: return PSCL_LL(10);
    }
#undef PSCL_LL
}
