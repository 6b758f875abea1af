// scl128_spec.hip -- scl128_kernel instances with a compiled-in information set (CODE 1:
// construct_info_set(128, 64), CODE 2: construct_info_set(128, 88); scl128_impl.h).  All 128
// phases are unrolled with the frozen/info pattern known, so every per-phase branch on the
// information set and the info index fold away.  The build compiles this file once per
// (PSCL_SPEC_CODE, PSCL_SPEC_LMAX) pair so the large instances compile in parallel; each
// object defines pscl_launch_spec_<code>_<lmax>.
#include "scl128_impl.h"

#ifndef PSCL_SPEC_CODE
#error "PSCL_SPEC_CODE (1 or 2) and PSCL_SPEC_LMAX (1, 2, 4, 8) must be defined"
#endif

#define PSCL_SPEC_CAT2(a, b, c) pscl_launch_spec_##a##_##b
#define PSCL_SPEC_CAT(a, b) PSCL_SPEC_CAT2(a, b, 0)
#define PSCL_SPEC_FN PSCL_SPEC_CAT(PSCL_SPEC_CODE, PSCL_SPEC_LMAX)

// (128,64) decodes read plain channel rows; (128,88) is the NR code, decoded rate matched
hipError_t PSCL_SPEC_FN(const pscl_decode_params& P, bool fs, int wpg, int64_t grid, int lds, hipStream_t s) {
    constexpr bool CH = PSCL_SPEC_CODE == 2;
    if (P.apx && !fs)  // screening decode (plain decodes)
        hipLaunchKernelGGL((scl128_kernel<PSCL_SPEC_LMAX, false, CH, false, PSCL_SPEC_CODE, true>), dim3((unsigned)grid),
                           dim3(wpg * 64), lds, s, P);
#if PSCL_SPEC_CODE == 1 && PSCL_SPEC_LMAX >= 4
    else if (P.apx && fs)  // screening decode with forced bits (the DL-SCL retry rounds)
        hipLaunchKernelGGL((scl128_kernel<PSCL_SPEC_LMAX, false, CH, true, PSCL_SPEC_CODE, true>), dim3((unsigned)grid),
                           dim3(wpg * 64), lds, s, P);
#endif
    else if (fs)
        hipLaunchKernelGGL((scl128_kernel<PSCL_SPEC_LMAX, false, CH, true, PSCL_SPEC_CODE>), dim3((unsigned)grid),
                           dim3(wpg * 64), lds, s, P);
    else
        hipLaunchKernelGGL((scl128_kernel<PSCL_SPEC_LMAX, false, CH, false, PSCL_SPEC_CODE>), dim3((unsigned)grid),
                           dim3(wpg * 64), lds, s, P);
    return hipGetLastError();
}
