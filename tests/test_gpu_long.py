"""GPU: code lengths above 128 (csrc/scl_long.hip).  The reference's decode_scl accepts any
power-of-two N (dl_scl_polar/polar/scl.py:25-30); these tests hold the long-code kernel to
the reference's own outputs at N = 256, 512 and 1024 (tests/golden/g14_*.npz, made by
tests/golden/make_golden.py g14) and to the oracle on larger random sets -- candidates, list
order, path counts, fp64 metrics and decision LLRs bit for bit."""
import numpy as np
import pytest

import oracle
from polar_code_amd import _native
from polar_code_amd.polar.crc import attach_crc
from polar_code_amd.polar.polar import _polar_transform, construct_info_set
from polar_code_amd.polar.scl import decode_scl

pytestmark = pytest.mark.gpu
POLY = "0x1864CFB"


def _assert_decode(out, f, n, c, m, il, b, tag):
    assert out["n_paths"][f] == n, tag
    np.testing.assert_array_equal(out["cands"][f, :n], c[:n], err_msg=tag)
    np.testing.assert_array_equal(out["metrics"][f, :n], m[:n], err_msg=tag)
    np.testing.assert_array_equal(out["info_llrs"][f, :n], il[:n], err_msg=tag)
    assert out["best_idx"][f] == b, tag


@pytest.mark.parametrize("name", ["g14_n256", "g14_n256_forced", "g14_n512", "g14_n1024"])
def test_long_codes_match_reference_golden(golden, name):
    g = golden(f"{name}.npz")
    crc = str(g["crc"]) or None
    info = g["info"]
    for key in g["keys"]:
        key = str(key)
        M = int(key.split("_")[0][1:])
        llr = g[key + "_llr"]
        force = g[key + "_force"]
        dec = _native.Decoder(llr.shape[1], info, M, crc)
        out = dec.decode(llr, None if np.all(force == -1) else force)
        for f in range(llr.shape[0]):
            _assert_decode(out, f, g[key + "_npaths"][f], g[key + "_cands"][f], g[key + "_metrics"][f],
                           g[key + "_info_llrs"][f], g[key + "_best"][f], f"{name} {key} frame {f}")
        # the reference API on one frame
        r = decode_scl(llr[0], info, M, crc=crc, force_info_bits=None if np.all(force[0] == -1) else force[0])
        np.testing.assert_array_equal(r["best_path_bits"], g[key + "_cands"][0][g[key + "_best"][0]])


def test_long_sc_decode_matches_reference_golden(golden):
    g = golden("g14_sc256.npz")
    dec = _native.Decoder(256, g["info"], 1, None)
    np.testing.assert_array_equal(dec.sc_decode(g["llr"]), g["bits"])


@pytest.mark.parametrize("N,K,M,ebno", [(256, 128, 8, 1.5), (512, 200, 16, 1.0), (1024, 512, 4, 1.0),
                                        (1024, 800, 32, 2.0), (256, 40, 3, 0.0)])
def test_long_codes_match_oracle(N, K, M, ebno):
    rng = np.random.default_rng(N + K + M)
    info = construct_info_set(N, K)
    B = 24
    msg = attach_crc(rng.integers(0, 2, size=(B, K - 24), dtype=np.int8), POLY)
    u = np.zeros((B, N), np.int8)
    u[:, info] = msg
    nv = 1.0 / (2.0 * K / N * 10 ** (ebno / 10))
    llr = 2.0 * ((1.0 - 2.0 * _polar_transform(u)) + rng.normal(0.0, np.sqrt(nv), size=(B, N))) / nv
    llr[:4] = np.round(llr[:4])  # integer LLRs: exact metric ties through the stable sort
    dec = _native.Decoder(N, info, M, POLY)
    out = dec.decode(llr)
    plain = dec.decode(llr, want_metrics=False, want_cands=False, want_info_llrs=False)
    for f in range(B):
        n, c, m, il, b = oracle.decode_scl(llr[f], info, M, crc=POLY)
        _assert_decode(out, f, n, c, m, il, b, f"N={N} M={M} frame {f}")
        np.testing.assert_array_equal(plain["best_bits"][f], c[b])
        assert bool(plain["crc_pass"][f]) == oracle.check_crc(c[b], POLY)


def test_long_decode_with_retries_matches_oracle():
    """DL-SCL (flip.py:65-141, beta None) at N = 256: the batched retry loop (forced decodes
    with decision LLRs on the long-code kernel) against the oracle, frame by frame."""
    from polar_code_amd.dlscl.flip import decode_with_retries_batch

    N, K, M, retries = 256, 128, 4, 6
    rng = np.random.default_rng(77)
    info = construct_info_set(N, K)
    B = 40
    msg = attach_crc(rng.integers(0, 2, size=(B, K - 24), dtype=np.int8), POLY)
    u = np.zeros((B, N), np.int8)
    u[:, info] = msg
    nv = 1.0 / (2.0 * K / N * 10 ** (3.5 / 10))
    llr = 2.0 * ((1.0 - 2.0 * _polar_transform(u)) + rng.normal(0.0, np.sqrt(nv), size=(B, N))) / nv
    out = decode_with_retries_batch(llr, info, M, retries, crc=POLY)
    assert np.count_nonzero(out["attempts"] > 1) >= 3  # some frames exercise the retry loop
    for f in range(B):
        r = oracle.decode_with_retries(llr[f], info, M, retries, crc=POLY)
        np.testing.assert_array_equal(out["best_bits"][f], r["bits"], err_msg=f"frame {f}")
        assert bool(out["success"][f]) == r["success"] and out["attempts"][f] == r["attempts"], f
        assert [int(t) for t in out["tried"][f] if t >= 0] == r["tried"], f


@pytest.mark.parametrize("N,K,M,retries,use_beta,snr,chunks", [(256, 128, 4, 6, False, 2.0, "1"),
                                                             (256, 128, 8, 4, True, 1.5, "2"),
                                                             (512, 256, 4, 3, False, 1.25, "1")])
def test_long_device_retry_loop(N, K, M, retries, use_beta, snr, chunks):
    """The device DL-SCL loop at N > 128 (HIST long-kernel retry decodes, dense per-round state)
    equals the host-ranked batch form frame by frame (bits, CRC, attempts, tried indices) and
    the oracle on a sample; in-kernel counters match the host's counts."""
    from polar_code_amd.dlscl.flip import decode_with_retries_batch, decode_with_retries_device

    rng = np.random.default_rng(N + K + M)
    info = construct_info_set(N, K)
    B = 600
    msg = attach_crc(rng.integers(0, 2, size=(B, K - 24), dtype=np.int8), POLY)
    u = np.zeros((B, N), np.int8)
    u[:, info] = msg
    nv = 1.0 / (2.0 * K / N * 10 ** (snr / 10))
    llr = 2.0 * ((1.0 - 2.0 * _polar_transform(u)) + rng.normal(0.0, np.sqrt(nv), size=(B, N))) / nv
    beta = rng.random((K, K)).astype(np.float32) if use_beta else None  # (the reference stores beta in fp32)
    dev = decode_with_retries_device(llr, info, M, retries, crc=POLY, beta=beta, msg=msg,
                                     tuning={"dl_chunks": int(chunks)})
    host = decode_with_retries_batch(llr, info, M, retries, crc=POLY, beta=beta)
    assert np.count_nonzero(host["attempts"] > 1) >= 50  # the retry loop is exercised
    for k in ("best_bits", "success", "attempts", "tried"):
        np.testing.assert_array_equal(dev[k], host[k], err_msg=k)
    cd = dev["counters"]["dl"]
    assert cd[_native.CNT_FRAME_ERR] == int(np.count_nonzero(~host["success"]))
    assert cd[_native.CNT_BIT_ERR] == int(np.count_nonzero(host["best_bits"] != msg))
    assert cd[_native.CNT_RETRIES] == int((host["attempts"] - 1).sum())
    for f in range(0, B, 40):  # the reference loop (oracle) on a sample
        r = oracle.decode_with_retries(llr[f], info, M, retries, crc=POLY, beta=beta)
        np.testing.assert_array_equal(dev["best_bits"][f], r["bits"], err_msg=f"frame {f}")
        assert dev["attempts"][f] == r["attempts"], f
        assert [int(t) for t in dev["tried"][f] if t >= 0] == r["tried"], f


def test_long_device_counters():
    """Device-buffer decode with in-kernel FER/BER counting at N = 512."""
    N, K, M = 512, 256, 4
    rng = np.random.default_rng(5)
    info = construct_info_set(N, K)
    B = 300
    msg = attach_crc(rng.integers(0, 2, size=(B, K - 24), dtype=np.int8), POLY)
    u = np.zeros((B, N), np.int8)
    u[:, info] = msg
    nv = 1.0 / (2.0 * K / N * 10 ** (1.0 / 10))
    llr = 2.0 * ((1.0 - 2.0 * _polar_transform(u)) + rng.normal(0.0, np.sqrt(nv), size=(B, N))) / nv
    dec = _native.Decoder(N, info, M, POLY)
    W = dec.W
    words = np.zeros((B, W), np.uint64)
    for jj in range(K):
        words[:, jj >> 6] |= msg[:, jj].astype(np.uint64) << np.uint64(jj & 63)
    host = dec.decode(llr, want_metrics=False, want_cands=False, want_info_llrs=False)
    with _native.DeviceArena(dec) as mem:
        d_llr, d_ref = mem.alloc(llr.nbytes), mem.alloc(words.nbytes)
        d_best, d_flags, d_cnt = mem.alloc(B * W * 8), mem.alloc(B), mem.alloc(64)
        mem.upload(d_llr, llr)
        mem.upload(d_ref, words)
        mem.memset(d_cnt, 0, 64)
        dec.decode_device(d_llr, B, d_best=d_best, d_flags=d_flags, d_ref=d_ref, k_payload=K - 24, d_counters=d_cnt)
        dec.sync()
        cnt = mem.download(d_cnt, 64, np.int64)
        flags = mem.download(d_flags, B, np.uint8)
    assert cnt[0] == B
    assert cnt[1] == int(np.count_nonzero(~host["crc_pass"]))
    assert cnt[2] == int(np.count_nonzero(host["best_bits"] != msg))
    np.testing.assert_array_equal((flags & 0x80) != 0, host["crc_pass"])


@pytest.mark.parametrize("N,E", [(256, 300), (256, 200), (512, 600)])
def test_long_code_rate_matched_staging(N, E):
    """The long-code kernel's rate-matched channel staging (de-repetition / de-puncture and
    sub-block de-interleave fused into the staging, pscl_set_rate_match with N > 128) against the
    package's host mirrors of scl_nr.py:47-48 plus the oracle, every output bit for bit."""
    from polar_code_amd.nr.polar import derate_match_polar, subblock_deinterleave

    rng = np.random.default_rng(N + E)
    K = N // 2
    info = construct_info_set(N, K)
    llrE = rng.normal(1.5, 3.0, size=(40, E))
    llrE[:5] = np.round(llrE[:5])  # integer LLRs: exact metric ties through the front end
    dec = _native.Decoder(N, info, 4, POLY)
    dec.set_rate_match(E)
    out = dec.decode(llrE)
    internal = np.stack([subblock_deinterleave(derate_match_polar(x, N), N) for x in llrE])
    for f in range(llrE.shape[0]):
        n, c, m, il, b = oracle.decode_scl(internal[f], info, 4, crc=POLY)
        _assert_decode(out, f, n, c, m, il, b, f"N={N} E={E} frame {f}")
