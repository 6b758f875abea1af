// scl128.hip -- launches of the specialised N = 128, L <= 8 list decoder (scl128_impl.h).
// The general instances (any information set, decision history, rate matching) live here;
// the BASELINE codes' compiled-in instances come from scl128_spec.hip objects.
#include "scl128_impl.h"

#define PSCL_SPEC_DECL(c, l) \
    hipError_t pscl_launch_spec_##c##_##l(const pscl_decode_params& P, bool fs, int wpg, int64_t grid, int lds, hipStream_t s);
PSCL_SPEC_DECL(1, 1)
PSCL_SPEC_DECL(1, 2)
PSCL_SPEC_DECL(1, 4)
PSCL_SPEC_DECL(1, 8)
PSCL_SPEC_DECL(2, 1)
PSCL_SPEC_DECL(2, 2)
PSCL_SPEC_DECL(2, 4)
PSCL_SPEC_DECL(2, 8)

namespace {

template <int LMAX, bool HIST, bool CH, bool FS>
hipError_t launch128k(const pscl_decode_params& P, int wpg, int64_t grid, int lds, hipStream_t s) {
    hipLaunchKernelGGL((scl128_kernel<LMAX, HIST, CH, FS, 0>), dim3((unsigned)grid), dim3(wpg * 64), lds, s, P);
    return hipGetLastError();
}

int spec_code(const pscl_decode_params& P) {
    if (PSCL_ABLATE) return 0;  // diagnostic builds time the general kernel
    for (int c = 1; c < 3; ++c)
        if (P.K == kSpecK[c] && P.info_mask[0] == kSpecInfo[c][0] && P.info_mask[1] == kSpecInfo[c][1]) return c;
    return 0;
}

// Kernel choice: the decision-history variant (tests, info_llrs outputs) always takes the
// general form; plain decodes of the BASELINE codes take a compiled-in information set
// ((128,64) without rate matching, (128,88) with it), with or without forced bits.
template <int LMAX>
hipError_t launch128(const pscl_decode_params& P, int hist, int wpg, int64_t grid, int lds, hipStream_t s) {
    const bool fs = P.force || P.sc_hard;
    if (hist)
        return P.rm_E ? launch128k<LMAX, true, true, true>(P, wpg, grid, lds, s)
                      : launch128k<LMAX, true, false, true>(P, wpg, grid, lds, s);
    // (without forced bits the compiled-in kernels assume a full list, L == LMAX)
    const int code = (fs || P.L == LMAX) ? spec_code(P) : 0;
    if (code == 1 && !P.rm_E) {
        switch (LMAX) {
            case 1: return pscl_launch_spec_1_1(P, fs, wpg, grid, lds, s);
            case 2: return pscl_launch_spec_1_2(P, fs, wpg, grid, lds, s);
            case 4: return pscl_launch_spec_1_4(P, fs, wpg, grid, lds, s);
            default: return pscl_launch_spec_1_8(P, fs, wpg, grid, lds, s);
        }
    }
    if (code == 2 && P.rm_E) {
        switch (LMAX) {
            case 1: return pscl_launch_spec_2_1(P, fs, wpg, grid, lds, s);
            case 2: return pscl_launch_spec_2_2(P, fs, wpg, grid, lds, s);
            case 4: return pscl_launch_spec_2_4(P, fs, wpg, grid, lds, s);
            default: return pscl_launch_spec_2_8(P, fs, wpg, grid, lds, s);
        }
    }
    if (P.apx) return hipErrorInvalidValue;  // screening exists for the compiled-in codes only
    if (P.rm_E)
        return fs ? launch128k<LMAX, false, true, true>(P, wpg, grid, lds, s)
                  : launch128k<LMAX, false, true, false>(P, wpg, grid, lds, s);
    return fs ? launch128k<LMAX, false, false, true>(P, wpg, grid, lds, s)
              : launch128k<LMAX, false, false, false>(P, wpg, grid, lds, s);
}

}  // namespace


// the launch launch128 makes for a plain decode (no history, no forced bits) has a screening
// form: a compiled-in code in its own input mode with a full-size list
int pscl_screening_fs_available(const pscl_decode_params& P) {
    if (!P.fast || P.sc_hard || P.rm_E || P.L != pscl_decode_lmax(P.L) || P.L < 4) return 0;
    return spec_code(P) == 1;
}

// the screening launch of this plain decode runs the lane-per-path kernel (scl128_lane.hip):
// the (128,64) code on plain channel rows or the NR (128,88) code on rate-matched rows
// (PSCL_LANE_NR), L = 8 (and L = 4 unless PSCL_LANE4 = 0)
int pscl_lane_available(const pscl_decode_params& P) {
    if (!PSCL_LANE || !P.apx || P.no_lane || P.force || P.sc_hard || P.fidx || P.d_count || P.elist) return 0;
    if (P.L != 8 && (P.L != 4 || !PSCL_LANE4)) return 0;
    if (P.N != 128) return 0;
    const int code = spec_code(P);
    return (code == 1 && !P.rm_E) || (code == 2 && P.rm_E && PSCL_LANE_NR);
}

// a screened DL-SCL retry round (bucket lists, forced bits, warm start, deferred entries to
// bucket lists of their own) of the (128,64) code at L = 4, 8 runs the lane-per-path FS kernel
int pscl_lane_fs_available(const pscl_decode_params& P) {
    if (!PSCL_LANE_FS || !P.apx || P.no_lane || !P.force || P.sc_hard || !P.elist || !P.amb_elist || !P.fidx) return 0;
    if (!P.warm_metric || !P.warm_u || P.d_count || P.ref || P.rm_E || P.N != 128 || P.out_by_row) return 0;
    if (P.L != 8 && P.L != 4) return 0;
    return spec_code(P) == 1;
}

// an exact decode of the (128,64) code (or the rate-matched NR (128,88) code) at L = 4, 8 without
// metrics, candidates or decision LLRs runs the exact lane-per-path instance (P.lane_exact): plain
// frames (optionally listed by P.fidx / P.d_count, outputs at their rows), or a forced-bit retry
// round of the (128,64) code (bucket lists, warm start)
int pscl_lane_exact_available(const pscl_decode_params& P) {
    if (!P.lane_exact || P.apx || P.no_lane || P.sc_hard || P.tx || P.fpost || P.long_mode) return 0;
    if (P.metrics || P.cands || P.info_llrs || P.best_info_llrs) return 0;
    if (P.N != 128 || (P.L != 8 && P.L != 4)) return 0;
    const int code = spec_code(P);
    if (P.force)
        return code == 1 && P.elist && P.fidx && P.warm_metric && P.warm_u && !P.d_count && !P.ref && !P.rm_E && !P.out_by_row;
    if (P.elist) return 0;
    return (code == 1 && !P.rm_E) || (code == 2 && P.rm_E);
}

int pscl_screening_available(const pscl_decode_params& P) {
    if (!P.fast || P.force || P.sc_hard || P.L != pscl_decode_lmax(P.L)) return 0;
    const int code = spec_code(P);
    return (code == 1 && !P.rm_E) || (code == 2 && P.rm_E);
}

int pscl_fast128_fstride(int L, int ch) {
    switch (pscl_decode_lmax(L)) {
        case 1: return ch ? Layout128<1, true>::FSTRIDE : Layout128<1, false>::FSTRIDE;
        case 2: return ch ? Layout128<2, true>::FSTRIDE : Layout128<2, false>::FSTRIDE;
        case 4: return ch ? Layout128<4, true>::FSTRIDE : Layout128<4, false>::FSTRIDE;
        default: return ch ? Layout128<8, true>::FSTRIDE : Layout128<8, false>::FSTRIDE;
    }
}

hipError_t pscl_launch_decode128(const pscl_decode_params& P, int hist, int wpg, int64_t grid, int lds, hipStream_t s) {
    switch (pscl_decode_lmax(P.L)) {
        case 1: return launch128<1>(P, hist, wpg, grid, lds, s);
        case 2: return launch128<2>(P, hist, wpg, grid, lds, s);
        case 4: return launch128<4>(P, hist, wpg, grid, lds, s);
        case 8: return launch128<8>(P, hist, wpg, grid, lds, s);
        default: return hipErrorInvalidValue;
    }
}
