"""Host build of the device metric code (csrc/glibc_softplus.h) is bit-identical to the
platform libm exp/log1p and to numpy's logaddexp(0, v) -- the reference's metric."""
import ctypes as C
from pathlib import Path

import numpy as np

LIB = Path(__file__).resolve().parent.parent / "oracle" / "libsoftplus_host.so"


def _lib():
    L = C.CDLL(str(LIB))
    L.softplus_compare.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
    L.softplus_port_batch.argtypes = [C.c_void_p, C.c_int64, C.c_void_p]
    return L


def _inputs(n, seed=0):
    rng = np.random.default_rng(seed)
    parts = [
        rng.normal(0, 8, n),
        rng.uniform(-1100, 1100, n),
        rng.standard_normal(n) * 10.0 ** rng.uniform(-20, 3, n),
        np.array([0.0, -0.0, 1e-300, -1e-300, 5e-324, 708.0, -708.4, 745.2, -745.2, 1e6, -1e6, 511.99, 512.0,
                  1023.9, 1024.0, 2 ** -54, -(2 ** -54), 2 ** -29, 0.4142, np.log(2.0)]),
    ]
    u = rng.integers(0, 2 ** 63, n, dtype=np.int64).view(np.float64)
    parts.append(u[np.isfinite(u)])
    return np.ascontiguousarray(np.concatenate(parts))


def test_port_matches_libm():
    v = _inputs(400_000)
    be, bl, bs = (np.zeros(1, np.int64) for _ in range(3))
    _lib().softplus_compare(v.ctypes.data, v.size, be.ctypes.data, bl.ctypes.data, bs.ctypes.data)
    assert (be[0], bl[0], bs[0]) == (0, 0, 0)


def test_port_matches_numpy_logaddexp():
    v = _inputs(50_000, seed=1)
    v = v[np.abs(v) < 1e300]
    out = np.empty_like(v)
    _lib().softplus_port_batch(v.ctypes.data, v.size, out.ctypes.data)
    ref = np.array([float(np.logaddexp(0.0, float(x))) for x in v])
    np.testing.assert_array_equal(out.view(np.int64), ref.view(np.int64))


def apx_grid():
    """|v| grid for the screening tail: dense over the decoder's working range, the 708..745
    40..708 range (k = 58..1021: the fp32 scaling of t underflows and ldexp(q, -k) scales down), the
    708..745 range where exp(-|v|) goes subnormal, tiny and huge magnitudes, both signs."""
    parts = [np.arange(0.0, 40.0, 1e-4), np.arange(40.0, 708.0, 1e-2), np.arange(708.0, 745.2, 1e-3), 2.0 ** -np.arange(0.0, 80.0, 0.25),
             np.array([745.13, 745.14, 745.2, 746.0, 800.0, 1e3, 1e6, 2 ** -1074])]
    v = np.concatenate(parts)
    return np.ascontiguousarray(np.concatenate([v, -v[::7]]))


SCR_EPS = 6.0 * 2.0 ** -23  # glibc_softplus.h PSCL_SCR_EPS: proven relative bound of the screening tail


def tail_error_ok(exact, apx):
    """|apx - exact| <= PSCL_SCR_EPS * exact (+ one subnormal ulp where the tail underflows)."""
    return np.abs(apx - exact) <= SCR_EPS * exact + 2.0 ** -1074


def test_screening_tail_within_bound_host():
    """The screening tail (pscl_softplus_tail_scr, host form: libm exp2f, correctly rounded
    reciprocal) is within PSCL_SCR_EPS of the exact tail relatively on a dense grid."""
    v = apx_grid()
    ex, ap = np.empty_like(v), np.empty_like(v)
    L = _lib()
    L.softplus_tails_batch.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    L.softplus_tails_batch(v.ctypes.data, v.size, ex.ctypes.data, ap.ctypes.data)
    assert np.all(ex >= 0) and np.all(ap >= 0)
    ok = tail_error_ok(ex, ap)
    assert ok.all(), (v[~ok][:5], ex[~ok][:5], ap[~ok][:5])
    nrm = ex > 2.0 ** -1000  # normal range (subnormal tails: absolute bound above)
    rel = np.abs(ap - ex)[nrm] / ex[nrm]
    assert rel.max() < SCR_EPS / 2  # typical case: well inside the proven bound


def test_screening_polynomial_error_bound():
    """The atanh polynomial hard-coded in pscl_softplus_tail_scr (glibc_softplus.h) stays within
    the 0.06-unit (2^-23) approximation error its proof budgets, evaluated exactly (long double)
    on a dense grid of w = s^2 in [0, 1/9]; guards the coefficients against edits."""
    import re

    src = (Path(__file__).resolve().parent.parent / "polar_code_amd" / "csrc" / "glibc_softplus.h").read_text()
    body = src[src.index("PSCL_HD double pscl_softplus_tail_scr"):]
    body = body[:body.index("const float q")]
    coef = [float.fromhex(h) for h in re.findall(r"(0x[0-9a-f.]+p-?\d+)f", body)]
    assert len(coef) == 4 and "2.0f);" in body  # c4, c3, c2, c1; c0 = 2
    c = [2.0, coef[3], coef[2], coef[1], coef[0]]  # c0..c4
    w = np.linspace(0.0, 1.0, 200_001, dtype=np.longdouble) / 9
    exact = np.zeros_like(w)
    t = np.ones_like(w)
    for i in range(40):
        exact += 2 * t / (2 * i + 1)
        t *= w
    p = sum(np.longdouble(ci) * w ** i for i, ci in enumerate(c))
    err = float(np.max(np.abs(p / exact - 1))) / 2.0 ** -23
    assert err < 0.07, err
