/*
 * Bit-exact softplus for the SCL path metric, usable from host C and gfx950 device code.
 *
 * The reference updates a path metric with
 *     metric + float(np.logaddexp(0.0, v))          dl_scl_polar/polar/scl.py:102-105
 * and numpy's scalar logaddexp (npy_logaddexp) is
 *     x == y        -> x + LOGE2
 *     tmp = x - y > 0 -> x + log1p(exp(-tmp))
 *     else          -> y + log1p(exp(tmp))
 * with exp/log1p taken from the platform libm (glibc 2.35 on this image).  The list
 * decoder sorts on these metrics, so to make decisions bit-identical at ties and
 * near-ties the device must reproduce glibc's exp and log1p *bit for bit*:
 *
 *   exp   : glibc 2.35 __exp_fma (the ifunc chosen on any FMA+AVX2 host, which is the
 *           case for the survey container and the MI355X host). Table-driven, N=128,
 *           degree-5 polynomial; the fused multiply-adds below follow that variant's
 *           instruction sequence exactly, every other operation is unfused.
 *   log1p : glibc 2.35 dbl-64 s_log1p.c (fdlibm algorithm with glibc's split
 *           polynomial evaluation); no FMA in that build.
 *
 * The exp table is regenerated from mathematics by gen_exp_table.py.  Host parity of
 * this header against libm is tested in tests/test_softplus_host.py; device parity in
 * tests/test_gpu_parity.py.
 *
 * Contraction must stay OFF for this file (hipcc: the pragma below; gcc: -ffp-contract=off).
 */
#ifndef PSCL_GLIBC_SOFTPLUS_H
#define PSCL_GLIBC_SOFTPLUS_H

#include <math.h>
#include <stdint.h>
#include <string.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#if defined(__HIPCC__) || defined(__HIP__)
#define PSCL_HD __host__ __device__ __forceinline__
#else
#define PSCL_HD static inline
#endif

#ifdef __clang__
#pragma clang fp contract(off)
#endif

#define PSCL_EXP_TABLE_WORDS 256

/* PSCL_ANY(c): true if c holds in any lane of the wavefront (wave-uniform branch on the
 * device; plain c on the host).  Used to skip rarely needed branch-free sections. */
#if defined(__HIP_DEVICE_COMPILE__)
/* (ballot of the i1 itself: __any() takes an int and costs a select + compare per test) */
#define PSCL_ANY(c) (__builtin_amdgcn_ballot_w64((bool)(c)) != 0)
#define PSCL_RARE(c) __builtin_expect(__builtin_amdgcn_ballot_w64((bool)(c)) != 0, 0)
#else
#define PSCL_RARE(c) (c)
#define PSCL_ANY(c) (c)
#endif

/* n / d, correctly rounded, for operands the metric guarantees to be "nice": d in [1, 4),
 * n zero or of magnitude >= 2^-60.  On the device this is the compiler's own IEEE fp64
 * division sequence (reciprocal, two Newton steps, residual correction) without the
 * v_div_scale / v_div_fixup instructions, which are the identity for such operands (they
 * only rescale near the overflow/denormal range and patch special values). */
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ double pscl_div_nice(double n, double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double q = n * r;
    const double rem = __builtin_fma(-d, q, n);
    return __builtin_fma(rem, r, q);
}
#else
#define pscl_div_nice(n, d) ((n) / (d))
#endif

/* constants from glibc's __exp_data (N = 128) */
#define PSCL_EXP_INVLN2N 0x1.71547652b82fep0 * 128.0
#define PSCL_EXP_SHIFT 0x1.8p52
#define PSCL_EXP_NEGLN2HIN -0x1.62e42fefa0000p-8
#define PSCL_EXP_NEGLN2LON -0x1.cf79abc9e3b3ap-47
#define PSCL_EXP_C2 0x1.ffffffffffdbdp-2
#define PSCL_EXP_C3 0x1.555555555543cp-3
#define PSCL_EXP_C4 0x1.55555cf172b91p-5
#define PSCL_EXP_C5 0x1.1111167a4d017p-7

/* numpy's LOGE2 (npy_math.h NPY_LOGE2) */
#define PSCL_LOGE2 0.693147180559945309417232121458176568

PSCL_HD uint64_t pscl_asu64(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}

PSCL_HD double pscl_asf64(uint64_t u) {
    double x;
    memcpy(&x, &u, 8);
    return x;
}

PSCL_HD double pscl_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

/* exp(x), bit-identical to glibc 2.35 __exp_fma.  T = the 256-word table (exp_table.inc). */
PSCL_HD double pscl_exp(double x, const uint64_t* T) {
    uint64_t ix = pscl_asu64(x);
    uint32_t abstop = (uint32_t)(ix >> 52) & 0x7ff;
    if (abstop - 0x3c9u >= 0x3fu) {
        if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + x; /* |x| < 2^-54, also +-0 */
        if (abstop > 0x408u) {                               /* |x| >= 1024 */
            if (ix == 0xfff0000000000000ULL) return 0.0;     /* -inf */
            if (abstop == 0x7ffu) return 1.0 + x;            /* nan, +inf */
            if (ix >> 63) return 0.0;                        /* __math_uflow(0) */
            return pscl_asf64(0x7ff0000000000000ULL);        /* __math_oflow(0) */
        }
        abstop = 0; /* 512 <= |x| < 1024: handled by the special case below */
    }
    double kd = pscl_fma(x, PSCL_EXP_INVLN2N, PSCL_EXP_SHIFT);
    uint64_t ki = pscl_asu64(kd);
    kd = kd - PSCL_EXP_SHIFT;
    double r = pscl_fma(kd, PSCL_EXP_NEGLN2HIN, x);
    r = pscl_fma(kd, PSCL_EXP_NEGLN2LON, r);
    uint64_t idx = 2 * (ki & 127);
    uint64_t top = ki << 45;
    double p1 = pscl_fma(r, PSCL_EXP_C3, PSCL_EXP_C2);
    double tr = r + pscl_asf64(T[idx]); /* tail + r */
    uint64_t sbits = T[idx + 1] + top;
    double r2 = r * r;
    double p2 = pscl_fma(r, PSCL_EXP_C5, PSCL_EXP_C4);
    double t = pscl_fma(p1, r2, tr);
    double r4 = r2 * r2;
    double tmp = pscl_fma(r4, p2, t);
    if (abstop == 0) {
        if ((ki & 0x80000000ULL) == 0) {
            /* k > 0: exponent of scale may have overflowed */
            double scale = pscl_asf64(sbits - (1009ULL << 52));
            double y = pscl_fma(scale, tmp, scale);
            return y * 0x1p1009;
        }
        /* k < 0: subnormal range, rounded once (glibc specialcase) */
        double scale = pscl_asf64(sbits + (1022ULL << 52));
        double st = tmp * scale;
        double y = scale + st;
        if (y < 1.0) {
            double hi = y + 1.0;
            double lo = (scale - y) + st;
            lo = ((1.0 - hi) + y) + lo;
            y = (lo + hi) - 1.0;
            if (y == 0.0) y = 0.0;
        }
        return y * 0x1p-1022;
    }
    double scale = pscl_asf64(sbits);
    return pscl_fma(scale, tmp, scale);
}

/* log1p(x), bit-identical to glibc 2.35 (dbl-64 s_log1p.c, non-FMA build). */
PSCL_HD double pscl_log1p(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
                 Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
                 Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
                 Lp7 = 1.479819860511658591e-01;
    uint64_t ix = pscl_asu64(x);
    int32_t hx = (int32_t)(ix >> 32);
    int32_t ax = hx & 0x7fffffff;
    int32_t k = 1, hu = 0;
    double f = 0.0, c = 0.0;
    if (hx < 0x3FDA827A) {
        if (ax >= 0x3ff00000) { /* x <= -1 */
            if (x == -1.0) return -pscl_asf64(0x7ff0000000000000ULL);
            return pscl_asf64(0x7ff8000000000000ULL);
        }
        if (ax < 0x3e200000) { /* |x| < 2^-29 */
            if (ax < 0x3c900000) return x;
            return x - (x * x) * 0.5;
        }
        if (hx > 0 || hx <= (int32_t)0xbfd2bec3) {
            k = 0;
            f = x;
            hu = 1;
        }
    }
    if (hx >= 0x7ff00000) return x + x;
    if (k != 0) {
        double u;
        if (hx < 0x43400000) {
            u = 1.0 + x;
            hu = (int32_t)(pscl_asu64(u) >> 32);
            k = (hu >> 20) - 1023;
            c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
            c = c / u;
        } else {
            u = x;
            hu = (int32_t)(pscl_asu64(u) >> 32);
            k = (hu >> 20) - 1023;
            c = 0.0;
        }
        hu &= 0x000fffff;
        uint64_t lo = pscl_asu64(u) & 0xffffffffULL;
        if (hu < 0x6a09e) {
            u = pscl_asf64(((uint64_t)(uint32_t)(hu | 0x3ff00000) << 32) | lo);
        } else {
            k += 1;
            u = pscl_asf64(((uint64_t)(uint32_t)(hu | 0x3fe00000) << 32) | lo);
            hu = (0x00100000 - hu) >> 2;
        }
        f = u - 1.0;
    }
    double hfsq = (0.5 * f) * f;
    if (hu == 0) { /* |f| < 2^-20 */
        if (f == 0.0) {
            if (k == 0) return 0.0;
            double kd = (double)k;
            return (kd * ln2_lo + c) + kd * ln2_hi;
        }
        double R = (1.0 - 0.66666666666666666 * f) * hfsq;
        if (k == 0) return f - R;
        double kd = (double)k;
        return kd * ln2_hi - ((R - (kd * ln2_lo + c)) - f);
    }
    double s = f / (2.0 + f);
    double z = s * s;
    double z2 = z * z;
    double z4 = z2 * z2;
    double z6 = z2 * z4;
    double R = ((z * Lp1 + z2 * (z * Lp3 + Lp2)) + z4 * (z * Lp5 + Lp4)) + z6 * (z * Lp7 + Lp6);
    double sR = (R + hfsq) * s;
    if (k == 0) return f - (hfsq - sR);
    double kd = (double)k;
    return kd * ln2_hi - ((hfsq - ((kd * ln2_lo + c) + sR)) - f);
}

/*
 * Branch-free forms for the decoder's domain: exp(x) for x <= 0 and log1p(y) for y in [0, 1].
 * Every branch of the functions above is evaluated and the live one selected, so a wavefront
 * runs one straight-line sequence instead of exec-masked divergent regions.  Results are
 * identical to pscl_exp / pscl_log1p on that domain (tests/test_softplus_host.py).
 */
PSCL_HD double pscl_sel(bool c, double a, double b) { return c ? a : b; }

/* Device forms of three steps of the exp below, written out: fma(-|v|, s, c) with the sign
 * and magnitude as source modifiers, fma(a, s, c) as one VOP3 instead of a copy of the
 * constant addend plus v_fmac, and the high word of the scale, hi + (k << 13). */
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ double pscl_fma_negabs(double v, double s, double c) {
    double d;
    asm("v_fma_f64 %0, -|%1|, %2, %3" : "=v"(d) : "v"(v), "s"(s), "v"(c));
    return d;
}
__device__ __forceinline__ double pscl_fma3(double a, double s, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(s), "v"(c));
    return d;
}
__device__ __forceinline__ uint32_t pscl_shl13_add(uint32_t k, uint32_t hi) {
    uint32_t d;
    asm("v_lshl_add_u32 %0, %1, 13, %2" : "=v"(d) : "v"(k), "v"(hi));
    return d;
}
#else
#define pscl_fma_negabs(v, s, c) pscl_fma(-fabs(v), (s), (c))
#define pscl_fma3(a, s, c) pscl_fma((a), (s), (c))
#define pscl_shl13_add(k, hi) ((uint32_t)(hi) + ((uint32_t)(k) << 13))
#endif

/* exp(-|v|) */
PSCL_HD double pscl_exp_negabs(double v, const uint64_t* T) {
    const uint32_t abstop = (uint32_t)(pscl_asu64(v) >> 52) & 0x7ff;
    const double kd0 = pscl_fma_negabs(v, PSCL_EXP_INVLN2N, PSCL_EXP_SHIFT);
    const uint64_t ki = pscl_asu64(kd0);
    const double kd = kd0 - PSCL_EXP_SHIFT;
    double r = pscl_fma(kd, PSCL_EXP_NEGLN2HIN, -fabs(v));
    r = pscl_fma(kd, PSCL_EXP_NEGLN2LON, r);
    const uint64_t idx = 2 * (ki & 127);
    const double p1 = pscl_fma3(r, PSCL_EXP_C3, PSCL_EXP_C2);
    const double tr = r + pscl_asf64(T[idx]);
    /* sbits = T[idx+1] + (ki << 45): the shifted term has no low word, so only the high word
     * takes the sum (mod 2^32, as the 64-bit sum does mod 2^64) */
    const uint64_t tw = T[idx + 1];
    const uint32_t shi = pscl_shl13_add((uint32_t)ki, (uint32_t)(tw >> 32));
    const uint64_t sbits = ((uint64_t)shi << 32) | (uint32_t)tw;
    const double r2 = r * r;
    const double p2 = pscl_fma3(r, PSCL_EXP_C5, PSCL_EXP_C4);
    const double t = pscl_fma(p1, r2, tr);
    const double tmp = pscl_fma(r2 * r2, p2, t);
    /* main range */
    const double sc = pscl_asf64(sbits);
    double y = pscl_fma(sc, tmp, sc);
    if (PSCL_RARE(abstop - 0x3c9u >= 0x3fu)) {
        /* outside 2^-54 <= |v| < 512 (glibc's abstop test) */
        if (PSCL_ANY(abstop == 0x408u)) {
            /* 512 <= |v| < 1024, k < 0: glibc specialcase, rounded once into the subnormal range */
            const double scale = pscl_asf64(sbits + (1022ULL << 52));
            const double st = tmp * scale;
            const double y0 = scale + st;
            const double hi = y0 + 1.0;
            const double lo = ((1.0 - hi) + y0) + ((scale - y0) + st);
            double yr = (lo + hi) - 1.0;
            yr = yr == 0.0 ? 0.0 : yr;
            const double yspec = pscl_sel(y0 < 1.0, yr, y0) * 0x1p-1022;
            y = abstop == 0x408u ? yspec : y;
        }
        y = abstop > 0x408u ? 0.0 : y;            /* |v| >= 1024 and inf: underflow to +0 */
        y = abstop < 0x3c9u ? 1.0 - fabs(v) : y;  /* |v| < 2^-54 and +-0: 1 + x, x = -|v| */
    }
    return y;
}

/* exp(x) for x <= 0 */
PSCL_HD double pscl_exp_neg(double x, const uint64_t* T) { return pscl_exp_negabs(x, T); }

PSCL_HD double pscl_log1p_unit(double y) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
                 Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
                 Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
                 Lp7 = 1.479819860511658591e-01;
    const int32_t hx = (int32_t)(pscl_asu64(y) >> 32);
    /* y < 2^-29 (tiny metric tails, |llr| > ~20): x - x*x/2, or x below 2^-54 */
    const double tiny = hx < 0x3c900000 ? y : y - (y * y) * 0.5;
    if (!PSCL_ANY(hx >= 0x3e200000)) return tiny;
    const bool kp = hx >= 0x3FDA827A; /* 1 + y >= sqrt(2): reduce through u = 1 + y */
    int32_t k = 0, hu = 1;
    double c = 0.0, f = y;
    if (PSCL_ANY(kp)) {
        const double u = 1.0 + y;
        const int32_t hu0 = (int32_t)(pscl_asu64(u) >> 32);
        int32_t ku = (hu0 >> 20) - 1023;
        double cu = (ku > 0) ? 1.0 - (u - y) : y - (u - 1.0);
        cu = pscl_div_nice(cu, u); /* u in [1.41, 2], |cu| = 0 or >= 2^-54 */
        int32_t hum = hu0 & 0x000fffff;
        const uint64_t ulo = pscl_asu64(u) & 0xffffffffULL;
        const bool big = hum >= 0x6a09e;
        const double un = pscl_asf64(((uint64_t)(uint32_t)(hum | (big ? 0x3fe00000 : 0x3ff00000)) << 32) | ulo);
        ku += big ? 1 : 0;
        hum = big ? ((0x00100000 - hum) >> 2) : hum;
        k = kp ? ku : 0;
        c = kp ? cu : 0.0;
        hu = kp ? hum : 1;
        f = kp ? un - 1.0 : y;
    }
    const double hfsq = (0.5 * f) * f;
    /* general case */
    const double s = pscl_div_nice(f, 2.0 + f); /* 2 + f in [1.7, 2.5] */
    const double z = s * s;
    const double z2 = z * z;
    const double z4 = z2 * z2;
    const double z6 = z2 * z4;
    const double R = ((z * Lp1 + z2 * (z * Lp3 + Lp2)) + z4 * (z * Lp5 + Lp4)) + z6 * (z * Lp7 + Lp6);
    const double sR = (R + hfsq) * s;
    double res = f - (hfsq - sR);
    if (PSCL_ANY(k != 0)) {
        const double kd = (double)k;
        const double bk = kd * ln2_hi - ((hfsq - ((kd * ln2_lo + c) + sR)) - f);
        res = k == 0 ? res : bk;
        if (PSCL_RARE(hu == 0)) { /* |f| < 2^-20 */
            const double R0 = (1.0 - 0.66666666666666666 * f) * hfsq;
            const double a_f0 = k == 0 ? 0.0 : (kd * ln2_lo + c) + kd * ln2_hi;
            const double a_nz = k == 0 ? f - R0 : kd * ln2_hi - ((R0 - (kd * ln2_lo + c)) - f);
            res = hu == 0 ? (f == 0.0 ? a_f0 : a_nz) : res;
        }
    } else if (PSCL_RARE(hu == 0)) { /* k == 0 with |f| < 2^-20 */
        const double R0 = (1.0 - 0.66666666666666666 * f) * hfsq;
        res = hu == 0 ? (f == 0.0 ? 0.0 : f - R0) : res;
    }
    return hx < 0x3e200000 ? tiny : res;
}

/* branch-free L = log1p(exp(-|v|)) (identical to pscl_softplus_tail for finite v and +-inf) */
PSCL_HD double pscl_softplus_tail_bf(double v, const uint64_t* T) {
    return pscl_log1p_unit(pscl_exp_negabs(v, T));
}

/*
 * Screening tail for scl128_kernel<..., APX = true>: L = log1p(exp(-x)), x = |v|, to a proven
 * relative error below PSCL_SCR_EPS = 6 * 2^-23 (about 2^-20.4), mostly in fp32:
 *
 *   k = round(x log2 e), r2 = k - x log2 e (fp64: one fma with the exact product; |r2| <= 1/2,
 *                                    error < 2^-42 from the rounded log2 e for x <= 4096)
 *   u = e^-(x - k ln2) = 2^r2            fp32: cvt + v_exp_f32, u in [0.7, 1.42]
 *   t = u 2^-k = e^-x                    fp32 ldexp (exact while normal; tiny t only feeds s)
 *   log1p(t) = 2 atanh(s), s = t/(2 + t) in [0, 1/3]:
 *   log1p(t) = 2 s P(s^2) = 2^-k * [u * rcp(2 + t) * 2P(s^2)]     (2P: 5 terms, fp32 Horner)
 *   L = ldexp((double)q, -k), q = u * rcp(2 + t) * 2P(s^2)
 *
 * 2P(w) approximates 2 atanh(sqrt w)/sqrt w = sum_i 2 w^i/(2i + 1) on w in [0, 1/9] by the
 * relative-error minimax polynomial of degree 4 (Remez in 40-digit arithmetic, coefficients
 * rounded to fp32 and the rounding re-optimised by search; 2 exact): 0.060 units of 2^-23 with
 * the fp32 coefficients evaluated exactly, 0.56 including the fp32 Horner roundings (dense
 * 2e5-point grid).  The 7-term Taylor series it replaces needed two more dependent FMAs.
 *
 * Relative error of q, in units of 2^-23 (v_exp_f32 and v_rcp_f32 within 1 ulp, roundings
 * 2^-24 each): u 1.2 (exp 1, r2 rounding to fp32 0.18, r2's fp64 error 0.0), rcp 1 + its
 * argument 0.5 + t's error through 2 + t 0.4, P 0.82 (Horner roundings and the minimax error
 * 0.62, s^2 error x dP/dw 0.2), the two products 1: 5.0 < 6.  The
 * final cvt and ldexp are exact (until fp64 underflow, where the exact tail is subnormal too:
 * then the error is at most one ulp of the result).  x is clamped to 4096 (the exact tail is 0
 * above ~745.2; the clamp keeps k in int range) -- or, in pscl_softplus_tail_scr_nc, not
 * clamped by a caller that guarantees |v| < 2^30 (the L = 8 screening kernel: channel LLRs
 * below 2^22, larger or NaN frames deferred).
 *
 * With positive increments every screening path metric is within PSCL_SCR_EPS + N * 2^-53 of
 * the exact metric relatively (the tail error, plus the fp64 summation of at most N = 128
 * increments -- the screening kernels exist for N = 128 only -- which the exact metric also
 * carries, so two such terms enter the comparison), and the kernel trusts an ordering of two metrics only when
 * their high words (sign, exponent, 20 mantissa bits) differ by more than PSCL_SCR_H: then
 * the larger exceeds the smaller by at least PSCL_SCR_H * 2^-21 relatively (one high-word
 * unit is 2^-21..2^-20 of the value), which must beat the 2 * (PSCL_SCR_EPS + 2 * 128 * 2^-53)
 * the two metrics' errors can close -- checked at compile time below.  Tests: tests/test_softplus_host.py
 * (host form) and tests/test_gpu_screening.py (device form, pscl_softplus_tails_device).
 */
#define PSCL_SCR_TERMS 5
#define PSCL_SCR_EPS (6.0 / 8388608.0)
/* 8 units: 8 * 2^-21 = 3.8e-6 against 4 * (6 * 2^-23) = 2.9e-6.  Measured on MI355X (L = 8,
 * 5 dB, 1e6 frames): frames re-decoded 0.55 % at 16 units -> 0.32 % at 8, and more full-list
 * phases keep the better children without a rank (tools/screen_rate.py, tools/ab_bench.sh) */
#ifndef PSCL_SCR_H
#define PSCL_SCR_H 8
#endif
#ifdef __cplusplus
static_assert(PSCL_SCR_H / 2097152.0 >= 4.0 * (PSCL_SCR_EPS + 2.0 * 128.0 * 1.1102230246251565e-16),
              "screening margin PSCL_SCR_H does not cover twice the metric error (with 2x safety)");
#endif
#define PSCL_LN2HI 6.93147180369123816490e-01 /* 32 trailing zero bits: k * LN2HI exact */
#define PSCL_LN2LO 1.90821492927058770002e-10
#define PSCL_INVLN2 0x1.71547652b82fep0
#define PSCL_LOG2E_F 1.44269504088896341f

#if defined(__HIP_DEVICE_COMPILE__)
/* min(|v|, c): one v_min_f64 with the magnitude as a source modifier (fmin would add
 * canonicalising maxes for signalling NaNs) */
__device__ __forceinline__ double pscl_absmin(double v, double c) {
    double d;
    asm("v_min_f64 %0, |%1|, %2" : "=v"(d) : "v"(v), "s"(c));
    return d;
}
__device__ __forceinline__ float pscl_exp2_f32(float a) { return __builtin_amdgcn_exp2f(a); }
__device__ __forceinline__ float pscl_rcp_f32(float a) { return __builtin_amdgcn_rcpf(a); }
__device__ __forceinline__ double pscl_ldexp_f64(double a, int e) { return __builtin_amdgcn_ldexp(a, e); }
#else
#define pscl_absmin(v, c) (fabs(v) < (c) ? fabs(v) : (c))
#define pscl_exp2_f32(a) exp2f(a)
#define pscl_rcp_f32(a) (1.0f / (a))
#define pscl_ldexp_f64(a, e) ldexp((a), (e))
#endif

/* the screening tail of x = |v| without the clamp: valid while k = round(x log2 e) fits the
 * 32-bit exponent arithmetic, i.e. |v| < 2^30 (the result is then the clamped form's: both are
 * 0 above 745.2).  The decode kernel that uses it (PSCL_TAIL_ABS = 0 builds) defers every frame
 * where one lane's share of the channel magnitudes sums to 2^25 or more (2^24 per half-share at
 * L = 4), or to NaN: every tree LLR is then below 16 * 2^25 = 2^29 */
PSCL_HD double pscl_softplus_tail_scr_nc(double v) {
    const double x = fabs(v);
    const double kd0 = pscl_fma(-x, PSCL_INVLN2, PSCL_EXP_SHIFT); /* low word = -k */
    const int32_t nk = (int32_t)(uint32_t)pscl_asu64(kd0);
    const double kd = kd0 - PSCL_EXP_SHIFT;                      /* -k */
    const double r2 = pscl_fma(-x, PSCL_INVLN2, -kd);            /* k - x log2 e */
    const float u = pscl_exp2_f32((float)r2);                    /* e^-(x - k ln2) */
    const float t = ldexpf(u, nk);                               /* e^-x */
    const float rc = pscl_rcp_f32(2.0f + t);
    const float s = t * rc;
    const float w = s * s;
    /* 2 P(w): degree-4 minimax of sum_i 2 w^i / (2i + 1) on [0, 1/9] (see above), Horner */
    float p = fmaf(0x1.208bd0p-2f, w, 0x1.1e510ap-2f);
    p = fmaf(p, w, 0x1.99dae8p-2f);
    p = fmaf(p, w, 0x1.5554e4p-1f);
    p = fmaf(p, w, 2.0f);
    const float q = (u * rc) * p;
    return pscl_ldexp_f64((double)q, nk);
}

PSCL_HD double pscl_softplus_tail_scr(double v) { return pscl_softplus_tail_scr_nc(pscl_absmin(v, 4096.0)); }

/*
 * Screening tail with an ABSOLUTE error bound (round 4; the screening kernels' default,
 * PSCL_TAIL_ABS): L = log1p(exp(-x)), x = |v|, in seven instructions, all fp32 after the
 * conversion:
 *
 *   x32 = fl32(|v|)                     v_cvt_f32_f64 with |.| (inf for |v| > FLT_MAX)
 *   t   = 2^(-x32 log2 e)               v_mul_f32, v_exp_f32 (0 once the exponent passes -150)
 *   L   = log2(1 + t) ln 2              v_add_f32, v_log_f32, v_mul_f32, v_cvt_f64_f32
 *
 * Relative accuracy is lost (t's exponent carries fl32 roundings of x log2 e; 1 + t rounds to
 * 2^-24), but the error is small in absolute terms everywhere, which is all the ordering
 * certificates need: every comparison the screening pass makes involves a metric of at least
 * ln 2 (a worse child pays |lam| + L >= ln 2; two distinct paths diverged where one took a
 * worse child), and a metric is a sum of at most N = 128 increments, so its error is at most
 * 128 * PSCL_TAIL_ABS_DELTA plus the fp64 summation error (relative, N * 2^-53).  (The long-code
 * kernel, scl_lane_long.hip, scales the margin to its N: 2 N PSCL_TAIL_ABS_DELTA.)
 *
 * The bound is measured, not assumed: pscl_tail_abs_f32 is a function of the fp32 value x32
 * alone, and tools/tests scan EVERY non-negative fp32 x32 (2^31 - 2^23 values, +inf included) on
 * the device against the bit-exact glibc port (pscl_tail_abs_scan_device,
 * tests/test_gpu_screening.py::test_tail_abs_exhaustive_device): max |L(x32) - glibc(x32)|
 * = PSCL_TAIL_ABS_SCAN.  For fp64 x the conversion adds |x32 - x| * max|dL/dx| <=
 * 2^-24 x e^-x / (1 + e^-x) <= 0.2785 * 2^-24, and glibc(x32) vs glibc(x) one ulp each
 * (< 2^-52): PSCL_TAIL_ABS_DELTA bounds the sum.
 */
#ifndef PSCL_TAIL_ABS
#define PSCL_TAIL_ABS 1
#endif
#define PSCL_LOG2E_F32 1.44269504088896341f
#define PSCL_LN2_F32 0.693147180559945309f
/* upper bound of the exhaustive device scan: measured on MI355X 1.2338e-7 = 2.07 * 2^-24, at
 * x32 = 0.28314 (tests/test_gpu_screening.py, profiles/r04c_screening_tests.txt) */
#ifndef PSCL_TAIL_ABS_SCAN
#define PSCL_TAIL_ABS_SCAN (3.0 / 16777216.0)
#endif
#define PSCL_TAIL_ABS_DELTA (PSCL_TAIL_ABS_SCAN + 0.2785 / 16777216.0 + 2.0 * 2.220446049250313e-16)
/* certificate margin: two metrics' errors (2 * 128 * delta), rounded up */
#define PSCL_TAIL_ABS_MARGIN (2.0 * 128.0 * PSCL_TAIL_ABS_DELTA * 1.0001)

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ float pscl_log2_f32(float a) { return __builtin_amdgcn_logf(a); }
__device__ __forceinline__ float pscl_cvt_abs_f32(double v) {
    float r;
    asm("v_cvt_f32_f64 %0, |%1|" : "=v"(r) : "v"(v));
    return r;
}
#else
#define pscl_log2_f32(a) log2f(a)
#define pscl_cvt_abs_f32(v) ((float)fabs(v))
#endif

PSCL_HD float pscl_tail_abs_f32(float x32) {
    const float t = pscl_exp2_f32(x32 * -PSCL_LOG2E_F32);
    return pscl_log2_f32(1.0f + t) * PSCL_LN2_F32;
}
PSCL_HD double pscl_softplus_tail_abs(double v) { return (double)pscl_tail_abs_f32(pscl_cvt_abs_f32(v)); }

/*
 * The same tail in bits (round 5; the lane kernels' plain decodes, PSCL_LANE_BITS): with the LLR tree
 * computed in units of log2 e (the channel LLRs multiplied by LOG2E once, as they are loaded), the
 * metric increment logaddexp(0, -+v) / ln 2 = relu(-+v') + L2(|v'|), L2(y) = log2(1 + 2^-y), and
 *
 *   y32 = fl32(|v'|)                    v_cvt_f32_f64 with |.|
 *   L2  = log2(1 + 2^-y32)              v_exp_f32 (negation as a source modifier), v_add_f32,
 *                                       v_log_f32, v_cvt_f64_f32
 *
 * drops the two fp32 multiplies of pscl_tail_abs_f32.  Error, all in bits:
 *   * the fp32 evaluation: max over EVERY non-negative fp32 y32 of |L2(y32) - log1p(exp(-y32 ln 2)) /
 *     ln 2| (the glibc port in fp64), scanned on the device (pscl_tail2_scan_device,
 *     tests/test_gpu_screening.py::test_tail2_exhaustive_device) = PSCL_TAIL2_SCAN;
 *   * the conversion: |y32 - y| <= 2^-24 y and |dL2/dy| = 2^-y / (1 + 2^-y), so at most
 *     2^-24 max_y y 2^-y / (1 + 2^-y) < 0.41 * 2^-24;
 *   * the reference's own rounding of each increment (one ulp, < 2^-52 at these magnitudes);
 *   * the scaled tree itself: f is 1-Lipschitz in each argument and g rounds once, so a leaf
 *     computed from the scaled channel row differs from log2 e times the fp64 leaf of the exact
 *     decode by at most (2 n + 1) u S' (u = 2^-53, S' = the row's sum of scaled magnitudes, n =
 *     log2 N levels: (n + 1) u S' for the scaled tree against real arithmetic -- the scaling and
 *     n levels, each channel value under n g nodes -- and log2 e * n u S for the fp64 tree).  The
 *     kernels defer every frame where one lane's share of the row has scaled magnitudes summing to
 *     PSCL_TAIL2_CHAN_SUM_G(G) or more: 2^14 with G = 4 or 8 lanes per frame (G distinct shares, S' <
 *     2^17), 2^13 with G = 16 or 32 (16 distinct shares -- at G = 32 lanes p and p + 16 hold the same
 *     elements -- so again S' < 2^17).  That term is then below PSCL_TAIL2_TREE = 2^-31 per increment
 *     for every N <= 1024 (21 * 2^-53 * 2^17 < 2^-31).
 *     (h(x) = log2(1 + 2^-x) is 1-Lipschitz, so the error of an increment is at most the error of
 *     its LLR whichever child the LLR's sign names.)
 */
#define PSCL_LOG2E_F64 1.4426950408889634
/* upper bound of the exhaustive device scan: measured on MI355X 1.4155e-7 = 2.37 * 2^-24 bits, at
 * y32 = 0.93874 (tests/test_gpu_screening.py::test_tail2_exhaustive_device, profiles/r05g_scan.txt) */
#ifndef PSCL_TAIL2_SCAN
#define PSCL_TAIL2_SCAN (2.5 / 16777216.0)
#endif
#define PSCL_TAIL2_TREE (1.0 / 2147483648.0)
#define PSCL_TAIL2_DELTA (PSCL_TAIL2_SCAN + 0.41 / 16777216.0 + 2.0 * 2.220446049250313e-16 + PSCL_TAIL2_TREE)
/* certificate margin of the bits form: two metrics' errors (2 * 128 * delta), rounded up */
#define PSCL_TAIL2_MARGIN (2.0 * 128.0 * PSCL_TAIL2_DELTA * 1.0001)
/* per-lane bound on the sum of the scaled channel magnitudes a lane holds (else the frame is deferred):
 * G lanes per frame, at most 16 distinct shares, S' < 2^17 in every case (see above) */
#define PSCL_TAIL2_CHAN_SUM 16384.0
#define PSCL_TAIL2_CHAN_SUM_G(G) ((G) >= 16 ? 0.5 * PSCL_TAIL2_CHAN_SUM : PSCL_TAIL2_CHAN_SUM)

PSCL_HD float pscl_tail2_f32(float y32) { return pscl_log2_f32(1.0f + pscl_exp2_f32(-y32)); }
PSCL_HD double pscl_softplus_tail2(double v) { return (double)pscl_tail2_f32(pscl_cvt_abs_f32(v)); }

/* L = log1p(exp(-|v|)), the part of logaddexp(0, +-v) shared by both bit hypotheses. */
PSCL_HD double pscl_softplus_tail(double v, const uint64_t* T) {
    double a = v < 0 ? -v : v;
    return pscl_log1p(pscl_exp(-a, T));
}

/* np.logaddexp(0.0, v) given the shared tail L (see above). */
PSCL_HD double pscl_logaddexp0(double v, double L) {
    if (v == 0.0) return PSCL_LOGE2; /* x == y branch: 0 + LOGE2 */
    return v > 0.0 ? v + L : 0.0 + L;
}

#endif /* PSCL_GLIBC_SOFTPLUS_H */
