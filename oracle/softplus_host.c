/*
 * TEST INFRASTRUCTURE: host build of polar_code_amd/csrc/glibc_softplus.h (the device
 * metric code) next to the platform libm, so tests/test_softplus_host.py can check the
 * port bit for bit on the CPU.  Not linked into the product.
 */
#include <math.h>
#include <stdint.h>

#include "glibc_softplus.h"

static const uint64_t kT[256] = {
#include "exp_table.inc"
};

/* count mismatches of (port exp, port log1p, port logaddexp0) vs libm over v[0..n) */
void softplus_compare(const double* v, int64_t n, int64_t* bad_exp, int64_t* bad_log1p, int64_t* bad_lae) {
    int64_t be = 0, bl = 0, bs = 0;
    for (int64_t i = 0; i < n; i++) {
        double x = -fabs(v[i]);
        double e1 = exp(x), e2 = pscl_exp(x, kT);
        if (pscl_asu64(e1) != pscl_asu64(e2)) be++;
        double l1 = log1p(e1), l2 = pscl_log1p(e1);
        if (pscl_asu64(l1) != pscl_asu64(l2)) bl++;
        /* npy_logaddexp(0, v) */
        double ref;
        if (v[i] == 0.0)
            ref = 0.0 + 0.693147180559945309417232121458176568;
        else if (0.0 - v[i] > 0)
            ref = 0.0 + log1p(exp(-(0.0 - v[i])));
        else
            ref = v[i] + log1p(exp(0.0 - v[i]));
        double got = pscl_logaddexp0(v[i], pscl_softplus_tail(v[i], kT));
        double got_bf = pscl_logaddexp0(v[i], pscl_softplus_tail_bf(v[i], kT));
        if (pscl_asu64(ref) != pscl_asu64(got) || pscl_asu64(ref) != pscl_asu64(got_bf)) bs++;
        if (pscl_asu64(pscl_exp_neg(x, kT)) != pscl_asu64(e1)) be++;
        if (pscl_asu64(pscl_log1p_unit(e1)) != pscl_asu64(l1)) bl++;
    }
    *bad_exp = be;
    *bad_log1p = bl;
    *bad_lae = bs;
}

void softplus_port_batch(const double* v, int64_t n, double* out) {
    for (int64_t i = 0; i < n; i++) out[i] = pscl_logaddexp0(v[i], pscl_softplus_tail_bf(v[i], kT));
}

/* log1p on [0, 1]: branch-free form vs libm */
int64_t log1p_unit_compare(const double* y, int64_t n) {
    int64_t bad = 0;
    for (int64_t i = 0; i < n; i++)
        if (pscl_asu64(pscl_log1p_unit(y[i])) != pscl_asu64(log1p(y[i]))) bad++;
    return bad;
}

/* exact and screening (bounded-error) metric tails, host forms */
void softplus_tails_batch(const double* v, int64_t n, double* exact, double* apx) {
    for (int64_t i = 0; i < n; i++) {
        exact[i] = pscl_softplus_tail_bf(v[i], kT);
        apx[i] = pscl_softplus_tail_scr(v[i]);
    }
}
