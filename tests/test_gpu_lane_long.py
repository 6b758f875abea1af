"""GPU: the runtime-information-set screening decoder (csrc/scl_lane_long.hip, N = 128..1024,
L = 4, 8, 16 and 32)
against the exact long-code kernel (scl_long.hip, screening off) and the oracle.

A plain decode (best bits and CRC flags only) of a long code runs the lane-per-path screening
kernel plus the exact re-decode of the frames it defers; its outputs must equal the exact
kernel's bit for bit (and, on a sample, the reference algorithm's: oracle.decode_scl, restating
dl_scl_polar/polar/scl.py:108-209).  Codes: construct_info_set(N, K) + CRC-24 at Eb/N0 points in
each code's waterfall (tools/long_bench.py), a K that is no multiple of 64, no CRC, integer LLRs
(exact metric ties: must be deferred), and huge / NaN-free extreme LLRs."""
import numpy as np
import pytest

import oracle
from polar_code_amd import _native
from polar_code_amd.polar.crc import attach_crc
from polar_code_amd.polar.polar import _polar_transform, construct_info_set

pytestmark = pytest.mark.gpu
POLY = "0x1864CFB"


def _frames(N, K, B, ebno, seed, crc=POLY):
    rng = np.random.default_rng(seed)
    info = construct_info_set(N, K)
    kp = K - 24 if crc else K
    msg = rng.integers(0, 2, size=(B, kp), dtype=np.int8)
    if crc:
        msg = attach_crc(msg, crc)
    u = np.zeros((B, N), np.int8)
    u[:, info] = msg
    nv = 1.0 / (2.0 * K / N * 10 ** (ebno / 10))
    llr = 2.0 * ((1.0 - 2.0 * _polar_transform(u)) + rng.normal(0.0, np.sqrt(nv), size=(B, N))) / nv
    return info, llr


def _screened_vs_exact(N, info, L, crc, llr):
    scr = _native.Decoder(N, info, L, crc)
    ex = _native.Decoder(N, info, L, crc)
    ex.set_screening(False)
    a = scr.decode(llr, want_metrics=False, want_cands=False, want_info_llrs=False)
    n_def = scr.screening_count()
    b = ex.decode(llr, want_metrics=False, want_cands=False, want_info_llrs=False)
    np.testing.assert_array_equal(a["best_bits"], b["best_bits"])
    np.testing.assert_array_equal(a["crc_pass"], b["crc_pass"])
    np.testing.assert_array_equal(a["best_idx"], b["best_idx"])
    np.testing.assert_array_equal(a["n_paths"], b["n_paths"])
    return a, n_def


@pytest.mark.parametrize("N,K,L,ebno,B", [(256, 128, 8, 4.0, 6000), (256, 128, 4, 4.0, 6000),
                                          (512, 256, 8, 5.0, 3000), (512, 256, 4, 5.0, 3000),
                                          (1024, 512, 8, 6.0, 1500), (1024, 512, 4, 6.0, 1500),
                                          (256, 100, 8, 2.5, 3000), (512, 300, 8, 3.0, 1500),
                                          (256, 128, 16, 4.0, 3000), (1024, 512, 16, 6.0, 800),
                                          (128, 64, 16, 4.0, 6000), (512, 256, 16, 5.0, 1500),
                                          (128, 64, 32, 4.0, 3000), (256, 128, 32, 4.0, 1500),
                                          (1024, 512, 32, 6.0, 400)])
def test_lane_long_equals_exact(N, K, L, ebno, B):
    info, llr = _frames(N, K, B, ebno, seed=N * 7 + K + L)
    a, n_def = _screened_vs_exact(N, info, L, POLY, llr)
    print(f"N={N} K={K} L={L} {ebno} dB: {n_def} of {B} frames deferred ({100.0 * n_def / B:.3f} %), "
          f"FER {1.0 - a['crc_pass'].mean():.4f}")
    assert n_def < B // 4  # the screening pass decides most frames itself
    for f in range(0, B, B // 6):  # the reference algorithm on a sample
        n, c, m, il, bi = oracle.decode_scl(llr[f], info, L, crc=POLY)
        np.testing.assert_array_equal(a["best_bits"][f], c[bi], err_msg=f"frame {f}")
        assert bool(a["crc_pass"][f]) == oracle.check_crc(c[bi], POLY), f


@pytest.mark.parametrize("N,L", [(256, 8), (1024, 4)])
def test_lane_long_no_crc(N, L):
    info, llr = _frames(N, N // 4, 1000, 2.0, seed=N + L, crc=None)
    a, _ = _screened_vs_exact(N, info, L, None, llr)
    assert a["crc_pass"].all()
    for f in range(0, 1000, 250):
        n, c, m, il, bi = oracle.decode_scl(llr[f], info, L, crc=None)
        np.testing.assert_array_equal(a["best_bits"][f], c[bi], err_msg=f"frame {f}")


@pytest.mark.parametrize("N,L", [(256, 8), (512, 4), (256, 16), (128, 16), (128, 32), (512, 32)])
def test_lane_long_ties_and_extremes_defer(N, L):
    """Integer LLRs (exact metric ties through the stable sort), noiseless +-1 rows and rows with
    LLRs beyond 2^25 must reach the exact kernel; the outputs equal it everywhere."""
    info, llr = _frames(N, N // 2, 600, 1.5, seed=3 * N + L)
    llr[:200] = np.round(llr[:200])
    llr[200:300] = np.sign(llr[200:300])
    llr[300:320, 5] = 3.0e8
    a, n_def = _screened_vs_exact(N, info, L, POLY, llr)
    assert n_def >= 100  # the noiseless rows tie at every information phase
    for f in [0, 1, 200, 201, 300, 301]:
        n, c, m, il, bi = oracle.decode_scl(llr[f], info, L, crc=POLY)
        np.testing.assert_array_equal(a["best_bits"][f], c[bi], err_msg=f"frame {f}")


def test_lane_long_device_counters_equal_exact():
    """In-kernel FER/BER counting through the screening pass (certified frames counted by the
    lane kernel, deferred ones by the exact re-decode at their own rows) equals the exact run."""
    N, K, L, B = 256, 128, 8, 4000
    info, llr = _frames(N, K, B, 3.5, seed=11)
    rng = np.random.default_rng(11)
    msg = attach_crc(rng.integers(0, 2, size=(B, K - 24), dtype=np.int8), POLY)  # (same stream as _frames)
    counts = []
    for on in (True, False):
        dec = _native.Decoder(N, info, L, POLY)
        dec.set_screening(on)
        W = dec.W
        words = np.zeros((B, W), np.uint64)
        for jj in range(K):
            words[:, jj >> 6] |= msg[:, jj].astype(np.uint64) << np.uint64(jj & 63)
        with _native.DeviceArena(dec) as mem:
            d_llr, d_ref = mem.alloc(llr.nbytes), mem.alloc(words.nbytes)
            d_best, d_flags, d_cnt = mem.alloc(B * W * 8), mem.alloc(B), mem.alloc(64)
            mem.upload(d_llr, llr)
            mem.upload(d_ref, words)
            mem.memset(d_cnt, 0, 64)
            dec.decode_device(d_llr, B, d_best=d_best, d_flags=d_flags, d_ref=d_ref, k_payload=K - 24,
                              d_counters=d_cnt)
            dec.sync()
            counts.append((mem.download(d_cnt, 64, np.int64)[:5].copy(), mem.download(d_best, B * W * 8, np.uint64),
                           mem.download(d_flags, B, np.uint8)))
        dec.close()
    (c1, b1, f1), (c0, b0, f0) = counts
    np.testing.assert_array_equal(c1, c0)
    np.testing.assert_array_equal(b1, b0)
    np.testing.assert_array_equal(f1, f0)
    assert c1[0] == B and c1[1] > 0


@pytest.mark.parametrize("N,L", [(256, 8), (512, 4), (1024, 8), (256, 16), (1024, 16), (256, 32), (1024, 32)])
def test_lane_long_bits_domain_bound_deferred(N, L):
    """The long-code lanes decode in bits too (channel LLRs scaled by log2 e, glibc_softplus.h
    pscl_softplus_tail2) and defer a frame whose lane share (positions = p mod G, G = min(L, 16)
    distinct shares: at L = 32 lanes p and p + 16 hold the same elements) has scaled magnitudes
    summing to PSCL_TAIL2_CHAN_SUM_G(L) or more -- PSCL_TAIL2_CHAN_SUM at L <= 8, half of it at
    L = 16 and 32, so the frame's sum stays below 2^17 either way.  Rows scaled to straddle that
    bound decode exactly as the exact kernel, deferred or not."""
    from test_gpu_screening import _header_const

    B = {256: 3000, 512: 1500, 1024: 800}[N] // (1 if L <= 8 else 2 if L == 16 else 4)
    info, llr = _frames(N, N // 2, B, {256: 4.0, 512: 5.0, 1024: 6.0}[N], seed=9100 + N + L)
    rng = np.random.default_rng(N + L)
    G = min(L, 16)
    log2e = _header_const("PSCL_LOG2E_F64")
    bound = _header_const("PSCL_TAIL2_CHAN_SUM") * (0.5 if L >= 16 else 1.0)
    share = lambda x: np.abs(x).reshape(x.shape[0], N // G, G).sum(axis=1).max(axis=1) * log2e  # noqa: E731
    pick = np.arange(0, B, 2)
    llr[pick] *= (bound * np.exp2(rng.uniform(-1.0, 1.0, size=pick.size)) / share(llr[pick]))[:, None]
    a, n_def = _screened_vs_exact(N, info, L, POLY, llr)
    over = int(np.sum(share(llr) >= bound))
    assert over > B // 8 and n_def >= over, (over, n_def)


@pytest.mark.parametrize("K,L,ebno", [(32, 8, 1.5), (100, 8, 4.5), (32, 4, 1.5), (100, 4, 4.5), (64, 8, "custom"),
                                      (100, 16, 4.0)])
def test_lane_n128_runtime_info_set(K, L, ebno):
    """N = 128 codes without a compiled-in screening kernel (K other than 64 and 88, or K = 64 with
    another information set): the runtime-information-set lane kernel at n = 7 screens them.  Bit for
    bit the exact kernel's outputs; the reference algorithm on a sample; integer LLRs (exact metric
    ties) deferred -- which also shows that the screening pass ran."""
    B = 6000
    if ebno == "custom":  # K = 64 on every other position from 32 on: not construct_info_set(128, 64)
        rng = np.random.default_rng(5)
        info = np.sort(np.concatenate([np.arange(33, 128, 2), rng.choice(np.arange(32, 128, 2), 16, replace=False)]))
        _, llr = _frames(128, 64, B, 5.0, seed=11)
        msg = attach_crc(rng.integers(0, 2, size=(B, 40), dtype=np.int8), POLY)
        u = np.zeros((B, 128), np.int8)
        u[:, info] = msg
        nv = 1.0 / (2.0 * 0.5 * 10 ** (5.0 / 10))
        llr = 2.0 * ((1.0 - 2.0 * _polar_transform(u)) + rng.normal(0.0, np.sqrt(nv), size=(B, 128))) / nv
    else:
        info, llr = _frames(128, K, B, ebno, seed=128 * 7 + K + L)
    a, n_def = _screened_vs_exact(128, info, L, POLY, llr)
    assert n_def < B // 4
    for f in range(0, B, B // 6):
        n, c, m, il, bi = oracle.decode_scl(llr[f], info, L, crc=POLY)
        np.testing.assert_array_equal(a["best_bits"][f], c[bi], err_msg=f"frame {f}")
    ties = np.round(llr[:600] / 4.0)
    _, n_tie = _screened_vs_exact(128, info, L, POLY, ties)
    assert n_tie > 0
