"""GPU: the screening decode (include/polar_scl.h pscl_set_screening) against the exact kernel.

Plain decodes of the compiled-in codes run a pass with bounded-error metric tails that hands
every frame whose list ordering it cannot certify to the exact kernel.  Its outputs — decoded
bits, CRC flag, best index, path count, device-side FER/BER counters — must equal the exact
decode's bit for bit, including on inputs built to produce exact metric ties (integer and
noiseless LLRs), where the screening pass must defer to the exact kernel."""
import numpy as np
import pytest

import oracle
from polar_code_amd import _native
from polar_code_amd.polar import crc as pcrc
from polar_code_amd.polar.polar import _polar_transform, construct_info_set

pytestmark = pytest.mark.gpu
POLY = "0x1864CFB"


def _frames(rng, B, info, ebno_db, K=64):
    msg = pcrc.attach_crc(rng.integers(0, 2, size=(B, K - 24), dtype=np.int8), POLY)
    u = np.zeros((B, 128), np.int8)
    u[:, info] = msg
    nv = 1.0 / (2.0 * (K - 24) / 128 * 10 ** (ebno_db / 10))
    return 2.0 * ((1.0 - 2.0 * _polar_transform(u)) + rng.normal(0.0, np.sqrt(nv), size=(B, 128))) / nv


def _pair(N, info, M):
    scr, ex = _native.Decoder(N, info, M, POLY), _native.Decoder(N, info, M, POLY)
    ex.set_screening(False)
    return scr, ex


def _plain(dec, llr):
    return dec.decode(llr, want_metrics=False, want_cands=False, want_info_llrs=False)


def _assert_same(a, b, tag):
    for k in ("n_paths", "best_bits", "crc_pass", "best_idx"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=f"{tag}: {k}")


@pytest.mark.parametrize("M", [1, 2, 4, 8])
def test_screening_equals_exact_awgn(M):
    rng = np.random.default_rng(7100 + M)
    info = construct_info_set(128, 64)
    llr = np.concatenate([_frames(rng, 4000, info, s) for s in (0.0, 1.5, 3.0, 4.5, 6.0)])
    scr, ex = _pair(128, info, M)
    _assert_same(_plain(scr, llr), _plain(ex, llr), f"M={M}")


@pytest.mark.parametrize("M", [1, 2, 4, 8])
def test_screening_ties_defer_to_exact(M):
    """Integer-valued and noiseless LLRs: exact metric ties are common, so many frames must be
    deferred; the results still equal the exact kernel's and the oracle's."""
    rng = np.random.default_rng(7200 + M)
    info = construct_info_set(128, 64)
    B = 1200
    llr = rng.integers(-4, 9, size=(B, 128)).astype(np.float64)
    llr[: B // 3] = rng.choice([-2.0, -1.0, 1.0, 2.0, 3.0], size=(B // 3, 128))
    llr[B // 3: 2 * B // 3] = 50.0 * np.sign(_frames(rng, B // 3, info, 60.0))  # noiseless
    scr, ex = _pair(128, info, M)
    a = _plain(scr, llr)
    _assert_same(a, _plain(ex, llr), f"ties M={M}")
    for f in range(0, B, 7):
        n, c, m, il, b = oracle.decode_scl(llr[f], info, M, crc=POLY)
        assert a["n_paths"][f] == n and a["best_idx"][f] == b, f
        np.testing.assert_array_equal(a["best_bits"][f], c[b], err_msg=f"f={f}")


@pytest.mark.parametrize("M", [4, 8])
def test_screening_nr_rate_matched(M):
    from polar_code_amd.nr.polar import derate_match_polar, subblock_deinterleave

    rng = np.random.default_rng(7300 + M)
    info = construct_info_set(128, 88)
    E = 256
    llrE = rng.normal(2.0, 3.0, size=(3000, E)) * rng.choice([1.0, -1.0], size=(3000, E), p=[0.9, 0.1])
    scr, ex = _pair(128, info, M)
    for d in (scr, ex):
        d.set_rate_match(E)
    a = _plain(scr, llrE)
    _assert_same(a, _plain(ex, llrE), f"NR M={M}")
    for f in range(0, 3000, 50):
        internal = subblock_deinterleave(derate_match_polar(llrE[f], 128), 128)
        n, c, m, il, b = oracle.decode_scl(internal, info, M, crc=POLY)
        assert a["best_idx"][f] == b
        np.testing.assert_array_equal(a["best_bits"][f], c[b])


@pytest.mark.parametrize("K,E,M", [(64, 256, 4), (64, 100, 8), (88, 0, 8), (60, 0, 4), (64, 0, 3)])
def test_plain_decode_without_screening_form(K, E, M):
    """Codes and modes with no compiled-in screening kernel ((128,64) rate matched, (128,88)
    unmatched, other information sets, L below its power of two): plain outputs equal the
    oracle's.  Rate-matched rows and L = 3 run no screening pass; unmatched rows at L = 4 and 8
    are screened by the runtime-information-set lane kernel (scl_lane_long.hip at n = 7)."""
    from polar_code_amd.nr.polar import derate_match_polar, subblock_deinterleave

    rng = np.random.default_rng(7400 + K + E + M)
    info = construct_info_set(128, K)
    B = 600
    llr = (_frames(rng, B, info, 3.0, K=K) if not E
           else rng.normal(2.0, 3.0, size=(B, E)) * rng.choice([1.0, -1.0], size=(B, E), p=[0.9, 0.1]))
    dec = _native.Decoder(128, info, M, POLY)
    if E:
        dec.set_rate_match(E)
    a = _plain(dec, llr)
    if E or M not in (4, 8):
        assert dec.screening_count() == 0
    for f in range(0, B, 5):
        x = subblock_deinterleave(derate_match_polar(llr[f], 128), 128) if E else llr[f]
        n, c, m, il, b = oracle.decode_scl(x, info, M, crc=POLY)
        assert a["n_paths"][f] == n and a["best_idx"][f] == b, f
        np.testing.assert_array_equal(a["best_bits"][f], c[b], err_msg=f"f={f}")
        assert bool(a["crc_pass"][f]) == oracle.check_crc(c[b], POLY), f


def test_screening_device_counters_equal_exact():
    """Device path with in-kernel FER/BER counting (the bench's step): deferred frames are
    counted by the exact re-decode at their own rows, once."""
    info = construct_info_set(128, 64)
    B = 200_000
    out = {}
    for on in (True, False):
        dec = _native.Decoder(128, info, 8, POLY)
        dec.set_screening(on)
        with _native.DeviceArena(dec) as mem:
            d_llr, d_msg = mem.alloc(B * 128 * 8), mem.alloc(B * 8)
            d_best, d_flags, d_cnt = mem.alloc(B * 8), mem.alloc(B), mem.alloc(8 * 8)
            mem.memset(d_cnt, 0, 64)
            dec.channel_device(0, 3, 2.0, 0.5, 40, 0, B, d_llr, d_msg)
            # a quarter of the frames quantised to integers (ties -> deferred frames)
            llr = mem.download(d_llr, B * 128 * 8, np.float64).reshape(B, 128)
            llr[: B // 4] = np.round(llr[: B // 4] / 4.0)
            mem.upload(d_llr, llr)
            dec.decode_device(d_llr, B, d_best=d_best, d_flags=d_flags, d_ref=d_msg, k_payload=40, d_counters=d_cnt)
            dec.sync()
            out[on] = (mem.download(d_best, B * 8, np.uint64), mem.download(d_flags, B, np.uint8),
                       mem.download(d_cnt, 64, np.int64))
    for i, k in enumerate(("best", "flags", "counters")):
        np.testing.assert_array_equal(out[True][i], out[False][i], err_msg=k)
    assert out[True][2][0] == B


@pytest.mark.parametrize("M", [4, 8])
def test_screening_huge_llrs_deferred(M):
    """L >= 4: the screening tail runs without its |v| clamp (pscl_softplus_tail_scr_nc), valid
    while every tree LLR stays below 2^30, so a frame whose channel magnitudes sum to 2^25 or more
    over one lane's share is handed to the exact kernel: results equal the exact decode's and the
    oracle's."""
    rng = np.random.default_rng(7400 + M)
    info = construct_info_set(128, 64)
    B = 4000
    llr = _frames(rng, B, info, 4.0)
    big = np.arange(0, B, 9)
    vals = np.array([2.0 ** 22, -(2.0 ** 22), 1e7, -3e9, 1e15, 2.0 ** 22 - 1.0])
    llr[big, rng.integers(0, 128, size=big.size)] = vals[np.arange(big.size) % vals.size]
    scr, ex = _pair(128, info, M)
    a = _plain(scr, llr)
    _assert_same(a, _plain(ex, llr), "huge LLRs")
    assert scr.screening_count() >= int(np.sum(np.abs(llr).max(axis=1) >= 2.0 ** 25))
    for f in big[::5]:
        n, c, m, il, b = oracle.decode_scl(llr[f], info, M, crc=POLY)
        assert a["n_paths"][f] == n and a["best_idx"][f] == b, f
        np.testing.assert_array_equal(a["best_bits"][f], c[b], err_msg=f"f={f}")


@pytest.mark.parametrize("M", [4, 8])
def test_screening_bits_domain_bound_deferred(M):
    """The lane kernels' plain decodes compute the tree in units of log2 e (glibc_softplus.h,
    pscl_softplus_tail2) and defer every frame where one lane's 16 scaled channel magnitudes sum to
    PSCL_TAIL2_CHAN_SUM or more (the scaled tree's error bound).  Frames straddling that bound
    (strong, noiseless-like rows scaled so the per-lane sums cross it) decode exactly as the exact
    kernel and the oracle, deferred or not.  (A lane holds the row positions i = p mod L.)"""
    rng = np.random.default_rng(7500 + M)
    info = construct_info_set(128, 64)
    B = 6000
    llr = _frames(rng, B, info, 4.0)
    bound = _header_const("PSCL_TAIL2_CHAN_SUM") / _header_const("PSCL_LOG2E_F64")
    # rows scaled so the largest per-lane share (128 / L values) sits between 0.5 and 2 times the bound
    lanes = np.abs(llr).reshape(B, 128 // M, M).sum(axis=1).max(axis=1)
    scale = bound * np.exp2(rng.uniform(-1.0, 1.0, size=B)) / lanes
    pick = np.arange(0, B, 3)
    llr[pick] *= scale[pick, None]
    scr, ex = _pair(128, info, M)
    a = _plain(scr, llr)
    _assert_same(a, _plain(ex, llr), "bits-domain bound")
    over = np.abs(llr).reshape(B, 128 // M, M).sum(axis=1).max(axis=1) * _header_const("PSCL_LOG2E_F64") >= \
        _header_const("PSCL_TAIL2_CHAN_SUM")
    assert over.sum() > 500 and scr.screening_count() >= int(over.sum())
    for f in pick[::40]:
        n, c, m, il, b = oracle.decode_scl(llr[f], info, M, crc=POLY)
        assert a["n_paths"][f] == n and a["best_idx"][f] == b, f
        np.testing.assert_array_equal(a["best_bits"][f], c[b], err_msg=f"f={f}")


@pytest.mark.parametrize("M", [4, 8])
def test_pipelined_decodes_equal_stream_ordered(M):
    """pscl_set_pipelined: a stream of plain decodes whose exact re-decodes overlap the next
    call (alternate output buffers, as bench.py steps), then join: every batch's best bits and
    flags, and the accumulated counters, equal the stream-ordered decodes'; an entry point other
    than a pipelined decode (memcpy) orders the pending re-decodes first."""
    info = construct_info_set(128, 64)
    B, nb = 60_000, 5
    res = {}
    for pipe in (True, False):
        dec = _native.Decoder(128, info, M, POLY)
        dec.set_pipelined(pipe)
        with _native.DeviceArena(dec) as mem:
            d_llr = [mem.alloc(B * 128 * 8) for _ in range(nb)]
            d_msg = [mem.alloc(B * 8) for _ in range(nb)]
            d_out = [(mem.alloc(B * 8), mem.alloc(B)) for _ in range(nb)]
            d_cnt = mem.alloc(8 * 8)
            mem.memset(d_cnt, 0, 64)
            for i in range(nb):
                dec.channel_device(11, 30 + i, 1.5 + 0.5 * i, 0.5, 40, i * B, B, d_llr[i], d_msg[i])
            # ties in the last batch: many deferred frames
            llr = mem.download(d_llr[nb - 1], B * 128 * 8, np.float64).reshape(B, 128)
            mem.upload(d_llr[nb - 1], np.round(llr / 4.0))
            for i in range(nb):
                dec.decode_device(d_llr[i], B, d_best=d_out[i][0], d_flags=d_out[i][1], d_ref=d_msg[i],
                                  k_payload=40, d_counters=d_cnt)
            res[pipe] = ([(mem.download(b, B * 8, np.uint64), mem.download(f, B, np.uint8)) for b, f in d_out],
                         mem.download(d_cnt, 64, np.int64))
            assert dec.screening_count() > 0
        dec.close()
    for i in range(nb):
        np.testing.assert_array_equal(res[True][0][i][0], res[False][0][i][0], err_msg=f"best, batch {i}")
        np.testing.assert_array_equal(res[True][0][i][1], res[False][0][i][1], err_msg=f"flags, batch {i}")
    np.testing.assert_array_equal(res[True][1], res[False][1], err_msg="counters")
    assert res[True][1][0] == nb * B


@pytest.mark.parametrize("M", [1, 2, 4, 8])
def test_screening_boundary_ties_every_frame(M):
    """Crafted worst cases for the screening pass: exactly zero leaf LLRs (every child pays
    LOGE2: equal child metrics straddle list position L at every full-list info phase, and
    ds_permute leaves positions unclaimed) and sparse zeros among small integers.  Every such
    frame must be handed to the exact re-decode (count > 0) and every frame must equal the oracle."""
    rng = np.random.default_rng(7400 + M)
    info = construct_info_set(128, 64)
    B = 384
    llr = rng.integers(-3, 4, size=(B, 128)).astype(np.float64)
    llr[: B // 4] = 0.0                                           # all leaves exactly zero
    llr[B // 4: B // 2] *= rng.random((B // 4, 128)) < 0.5        # half the channel LLRs zero
    llr[B // 2: 3 * B // 4, :64] = 0.0                            # zero left half: zero depth-1 f outputs
    scr, ex = _pair(128, info, M)
    a = _plain(scr, llr)
    assert scr.screening_count() >= B // 4
    _assert_same(a, _plain(ex, llr), f"boundary ties M={M}")
    for f in range(B):
        n, c, m, il, b = oracle.decode_scl(llr[f], info, M, crc=POLY)
        assert a["n_paths"][f] == n and a["best_idx"][f] == b, f
        np.testing.assert_array_equal(a["best_bits"][f], c[b], err_msg=f"f={f}")
        assert bool(a["crc_pass"][f]) == oracle.check_crc(c[b], POLY), f


def _header_const(name):
    """A numeric #define of csrc/glibc_softplus.h, evaluated (the tests hold the kernel to the
    header's own constants, not to copies)."""
    import re
    from pathlib import Path

    src = (Path(_native.__file__).resolve().parent / "csrc" / "glibc_softplus.h").read_text()
    consts = {}
    for m in re.finditer(r"^#define (PSCL_\w+) (.+)$", src, re.M):
        consts[m.group(1)] = m.group(2).split("/*")[0].strip()
    expr = consts[name]
    for _ in range(4):
        expr = re.sub(r"PSCL_\w+", lambda k: "(" + consts[k.group(0)] + ")", expr)
    return float(eval(expr.replace("f", "") if name.endswith("F32") else expr))


def test_tail_abs_exhaustive_device():
    """The screening tail is a function of x32 = fl32(|v|) alone: its absolute error against
    the bit-exact glibc port over EVERY non-negative fp32 x32 (+inf included) stays within
    PSCL_TAIL_ABS_SCAN, the measured term of the margin's proof (glibc_softplus.h)."""
    dec = _native.Decoder(128, construct_info_set(128, 64), 8, POLY)
    err, x32 = dec.tail_abs_scan()
    scan = _header_const("PSCL_TAIL_ABS_SCAN")
    print(f"exhaustive fp32 scan: max |tail_abs - glibc| = {err:.4e} = 2^{np.log2(err):.3f} at x32 = {x32!r} "
          f"(bound {scan:.4e})")
    assert 0.0 < err <= scan
    # a one-value scan equals the kernels' own tail at that value (plumbing check)
    e2, x2 = dec.tail_abs_scan(0x3F800000, 0x3F800000)  # x32 = 1.0 only
    ex, ap = dec.softplus_tails(np.array([1.0]))
    assert e2 == abs(ap[0] - ex[0]) and x2 in (0.0, 1.0)


def test_tail2_exhaustive_device():
    """The bits form of the screening tail (the lane kernels' plain decodes) against
    log1p(exp(-y ln 2)) / ln 2 from the bit-exact glibc port, over EVERY non-negative fp32 y32:
    within PSCL_TAIL2_SCAN, the measured term of its margin (glibc_softplus.h); and the margin
    covers two metrics of 128 increments of PSCL_TAIL2_DELTA."""
    dec = _native.Decoder(128, construct_info_set(128, 64), 8, POLY)
    err, y32 = dec.tail_abs_scan(bits=True)
    scan = _header_const("PSCL_TAIL2_SCAN")
    print(f"exhaustive fp32 scan (bits): max |tail2 - glibc/ln2| = {err:.4e} = 2^{np.log2(err):.3f} at "
          f"y32 = {y32!r} (bound {scan:.4e})")
    assert 0.0 < err <= scan
    assert _header_const("PSCL_TAIL2_MARGIN") >= 2 * 128 * _header_const("PSCL_TAIL2_DELTA")


def test_screening_tail_within_bound_device():
    """The device forms of both metric tails (pscl_softplus_tails_device): the exact one is
    bit-identical to the host port (itself bit-identical to libm, test_softplus_host.py), the
    screening one (pscl_softplus_tail_abs: fp32 exp/log) stays within PSCL_TAIL_ABS_DELTA of it in
    absolute terms on a dense fp64 grid -- the per-increment bound the kernel's ordering margin
    PSCL_TAIL_ABS_MARGIN is built on."""
    import ctypes as C

    from test_softplus_host import _lib, apx_grid

    v = apx_grid()
    dec = _native.Decoder(128, construct_info_set(128, 64), 8, POLY)
    ex_d, ap_d = dec.softplus_tails(v)
    ex_h, ap_h = np.empty_like(v), np.empty_like(v)
    L = _lib()
    L.softplus_tails_batch.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    L.softplus_tails_batch(v.ctypes.data, v.size, ex_h.ctypes.data, ap_h.ctypes.data)
    np.testing.assert_array_equal(ex_d.view(np.int64), ex_h.view(np.int64))
    delta = _header_const("PSCL_TAIL_ABS_DELTA")
    err = np.abs(ap_d - ex_d)
    assert np.all(err <= delta), (v[err > delta][:5], ex_d[err > delta][:5], ap_d[err > delta][:5])
    margin = _header_const("PSCL_TAIL_ABS_MARGIN")
    assert margin >= 2 * 128 * delta
    print(f"screening tail: max absolute error {err.max():.3e} = 2^{np.log2(err.max()):.2f} "
          f"(delta 2^{np.log2(delta):.2f}, margin {margin:.3e})")
