"""GPU parity: the HIP decoder (through the C ABI) against the reference's golden vectors
and against the C oracle on larger seeded sets.  Everything is compared bit for bit:
candidate bits, list order, best index, path count, and the fp64 metrics / decision LLRs
(the metric is bit-exact by construction, see csrc/glibc_softplus.h, so the 1e-5 relative
tolerance north_star allows is not needed)."""
import numpy as np
import pytest

import oracle
from polar_code_amd import _native
from polar_code_amd.polar import crc as pcrc
from polar_code_amd.polar.polar import construct_info_set, sc_decode
from polar_code_amd.polar.scl import decode_scl, SCLDecoder

pytestmark = pytest.mark.gpu

DECODE_SETS = ["g4_decode.npz", "g6_forced.npz", "g10_n16.npz", "g10_n32.npz", "g10_n64_nocrc.npz",
               "g10_k88.npz", "g10_m16.npz", "g10_n8.npz", "g10_n4.npz", "g10_n2.npz"]
POLY = "0x1864CFB"


def _assert_batch(out, g, key, M):
    n = g[key + "_npaths"]
    np.testing.assert_array_equal(out["n_paths"], n, err_msg=key)
    for f in range(len(n)):
        k = n[f]
        np.testing.assert_array_equal(out["cands"][f, :k], g[key + "_cands"][f, :k], err_msg=f"{key} f{f}")
        np.testing.assert_array_equal(out["metrics"][f, :k], g[key + "_metrics"][f, :k], err_msg=f"{key} f{f}")
        np.testing.assert_array_equal(out["info_llrs"][f, :k], g[key + "_info_llrs"][f, :k], err_msg=f"{key} f{f}")
    np.testing.assert_array_equal(out["best_idx"], g[key + "_best"], err_msg=key)


@pytest.mark.parametrize("name", DECODE_SETS)
def test_decode_golden(golden, name):
    g = golden(name)
    crc = str(g["crc"]) or None
    for key in map(str, g["keys"]):
        M = int(key.split("_")[0][1:])
        force = g[key + "_force"] if key + "_force" in g.files else None
        dec = _native.get_decoder(int(g["N"]), g["info"], M, crc)
        out = dec.decode(g[key + "_llr"], force)
        _assert_batch(out, g, key, M)


def test_decode_ties_golden(golden):
    g = golden("g5_ties.npz")
    for key in map(str, g["keys"]):
        M = int(key.split("_M")[1])
        out = _native.get_decoder(128, g["info"], M, POLY).decode(g[key + "_llr"])
        _assert_batch(out, g, key, M)


def test_decode_scl_api_single_frame(golden):
    g = golden("g4_decode.npz")
    res = decode_scl(g["M8_snr3_llr"][0], g["info"], 8, crc=POLY)
    b = g["M8_snr3_best"][0]
    assert len(res["candidates"]) == 8 and isinstance(res["metrics"][0], float)
    np.testing.assert_array_equal(res["best_path_bits"], g["M8_snr3_cands"][0][b])
    np.testing.assert_array_equal(res["best_path_info_llrs"], g["M8_snr3_info_llrs"][0][b])
    with pytest.raises(ValueError):
        decode_scl(g["M8_snr3_llr"][0], g["info"], 0)
    with pytest.raises(ValueError):
        decode_scl(g["M8_snr3_llr"][0], g["info"], 4, force_info_bits=np.full(64, 2, np.int8))
    with pytest.raises(ValueError):
        decode_scl(g["M8_snr3_llr"][0][:100], g["info"], 4)


def test_sc_decode_golden(golden):
    g = golden("g9_sc.npz")
    np.testing.assert_array_equal(sc_decode(g["llr"], g["info"]), g["bits"])
    np.testing.assert_array_equal(sc_decode(g["llr"][3], g["info"]), g["bits"][3])


def _frames(rng, B, info, snr, N=128, crc=POLY):
    K = info.size
    deg = (int(crc, 16).bit_length() - 1) if crc else 0
    msg = rng.integers(0, 2, size=(B, K - deg), dtype=np.int8)
    if crc:
        msg = pcrc.attach_crc(msg, crc)
    u = np.zeros((B, N), np.int8)
    u[:, info] = msg
    from polar_code_amd.polar.polar import _polar_transform
    x = _polar_transform(u)
    nv = 1.0 / (2.0 * (K / N) * 10 ** (snr / 10))
    return 2.0 * ((1.0 - 2.0 * x) + rng.normal(0, np.sqrt(nv), size=(B, N))) / nv


@pytest.mark.parametrize("M", [1, 2, 3, 4, 8, 16, 32])
def test_decode_vs_oracle_random(M):
    rng = np.random.default_rng(100 + M)
    info = construct_info_set(128, 64)
    B = 600 if M <= 8 else 150
    llr = np.concatenate([_frames(rng, B // 3, info, s) for s in (1.0, 3.0, 5.0)])
    out = _native.get_decoder(128, info, M, POLY).decode(llr)
    for f in range(llr.shape[0]):
        n, c, m, il, b = oracle.decode_scl(llr[f], info, M, crc=POLY)
        assert out["n_paths"][f] == n
        np.testing.assert_array_equal(out["cands"][f, :n], c[:n], err_msg=f"M={M} f={f}")
        np.testing.assert_array_equal(out["metrics"][f, :n], m[:n], err_msg=f"M={M} f={f}")
        np.testing.assert_array_equal(out["info_llrs"][f, :n], il[:n], err_msg=f"M={M} f={f}")
        assert out["best_idx"][f] == b
        assert out["crc_pass"][f] == oracle.check_crc(c[b], POLY)


def test_forced_vs_oracle():
    rng = np.random.default_rng(7)
    info = construct_info_set(128, 64)
    llr = _frames(rng, 300, info, 2.0)
    force = np.full((300, 64), -1, np.int8)
    for f in range(300):
        i = rng.integers(0, 64)
        force[f, :i] = rng.integers(0, 2, size=i)
        force[f, i] = rng.integers(0, 2)
        if f % 7 == 0:
            force[f] = rng.integers(-1, 2, size=64)
    out = _native.get_decoder(128, info, 4, POLY).decode(llr, force)
    for f in range(300):
        n, c, m, il, b = oracle.decode_scl(llr[f], info, 4, crc=POLY, force=force[f])
        assert out["n_paths"][f] == n
        np.testing.assert_array_equal(out["cands"][f, :n], c[:n])
        np.testing.assert_array_equal(out["metrics"][f, :n], m[:n])
        np.testing.assert_array_equal(out["info_llrs"][f, :n], il[:n])
        assert out["best_idx"][f] == b


def test_metric_softplus_probe():
    """N=2, K=1 exposes the metric directly: metrics = softplus(-f) + softplus(+-g).  Wide
    LLR magnitudes exercise every branch of the glibc exp/log1p port on the device."""
    rng = np.random.default_rng(11)
    B = 60000
    mag = 10.0 ** rng.uniform(-18, 3.1, size=(B, 2))
    llr = mag * rng.choice([-1.0, 1.0], size=(B, 2))
    llr[:100] = rng.integers(-3, 4, size=(100, 2)).astype(float)  # exact zeros and ties
    llr[100:200, 0] = -llr[100:200, 1]                             # g = 0 exactly
    out = _native.get_decoder(2, [1], 2, None).decode(llr)
    ref = np.empty((B, 2))
    for f in range(B):
        n, c, m, il, b = oracle.decode_scl(llr[f], np.array([1], np.int32), 2)
        ref[f] = m[:2]
    np.testing.assert_array_equal(out["metrics"].view(np.int64), ref.view(np.int64))


def test_scl_decoder_batch_and_device_api():
    import torch

    rng = np.random.default_rng(3)
    info = construct_info_set(128, 64)
    llr = _frames(rng, 1000, info, 3.0)
    dec = SCLDecoder(128, info, 8, POLY)
    host = dec.decode(llr)
    bits, ok = oracle.decode_batch(llr, info, 8, POLY)
    np.testing.assert_array_equal(host["bits"], bits)
    np.testing.assert_array_equal(host["crc_pass"], ok)
    t = torch.from_numpy(llr).cuda()
    words, flags = dec.decode_tensor(t)
    torch.cuda.synchronize()
    w = words.cpu().numpy().view(np.uint64)[:, 0]
    dev_bits = ((w[:, None] >> np.arange(64, dtype=np.uint64)) & 1).astype(np.int8)
    np.testing.assert_array_equal(dev_bits, bits)
    np.testing.assert_array_equal((flags.cpu().numpy() & 0x80) != 0, ok)


@pytest.mark.parametrize("N,K,L,E", [(128, 64, 8, 0), (128, 64, 4, 0), (64, 40, 4, 0), (32, 20, 2, 0),
                                     (128, 88, 2, 0), (16, 8, 16, 0), (128, 64, 8, 200), (128, 64, 2, 300)])
def test_path_llr_replay_equals_decoder_history(N, K, L, E):
    """pscl_path_llrs_device (replay from a path's bits) == the decoder's info_llrs, bit for bit."""
    rng = np.random.default_rng(N * 1000 + K + L + E)
    info = construct_info_set(N, K)
    B = 600
    llr = rng.normal(1.0, 2.5, size=(B, E or N)) * rng.choice([1.0, -1.0], size=(B, E or N))
    dec = _native.Decoder(N, info, L, "0x1864CFB" if K > 24 else None)
    if E:
        dec.set_rate_match(E)
    out = dec.decode(llr, want_metrics=False)
    rows = np.repeat(np.arange(B), L)
    valid = (np.arange(L)[None, :] < out["n_paths"][:, None]).ravel()
    cands = out["cands"].reshape(B * L, K)[valid]
    got = dec.path_llrs(llr[rows[valid]], cands)
    want = out["info_llrs"].reshape(B * L, K)[valid]
    np.testing.assert_array_equal(got.view(np.uint64), want.view(np.uint64))


@pytest.mark.parametrize("M", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("forced", [False, True])
def test_compiled_info_set_kernels_vs_oracle(M, forced):
    """Decodes without decision history of the BASELINE (128,64) code run the kernels with the
    information set compiled in (csrc/scl128_spec.hip), with and without forced bits; every
    candidate, fp64 metric, path count and best index against the oracle, bit for bit."""
    rng = np.random.default_rng(500 + M + 10 * forced)
    info = construct_info_set(128, 64)
    B = 900
    llr = np.concatenate([_frames(rng, B // 3, info, s) for s in (1.0, 3.0, 5.0)])
    force = None
    if forced:
        force = np.full((B, 64), -1, np.int8)
        for f in range(0, B, 2):
            i = rng.integers(0, 64)
            force[f, :i] = rng.integers(0, 2, size=i)
            force[f, i] = rng.integers(0, 2)
    out = _native.get_decoder(128, info, M, POLY).decode(llr, force, want_info_llrs=False)
    for f in range(B):
        n, c, m, il, b = oracle.decode_scl(llr[f], info, M, crc=POLY, force=None if force is None else force[f])
        assert out["n_paths"][f] == n, f
        np.testing.assert_array_equal(out["cands"][f, :n], c[:n], err_msg=f"M={M} f={f}")
        np.testing.assert_array_equal(out["metrics"][f, :n].view(np.int64), m[:n].view(np.int64))
        assert out["best_idx"][f] == b
        np.testing.assert_array_equal(out["best_bits"][f], c[b])


@pytest.mark.parametrize("M", [2, 8])
@pytest.mark.parametrize("E", [100, 256, 300])
def test_compiled_nr_kernels_vs_oracle(M, E):
    """The (128,88) NR code with rate matching runs the compiled-in kernels (CODE 2); metrics
    and candidates against the oracle decoding the host front-end's internal LLRs."""
    from polar_code_amd.nr.polar import derate_match_polar, subblock_deinterleave

    rng = np.random.default_rng(E + M)
    info = construct_info_set(128, 88)
    llrE = rng.normal(2.0, 3.0, size=(300, E)) * rng.choice([1.0, -1.0], size=(300, E), p=[0.9, 0.1])
    dec = _native.Decoder(128, info, M, POLY)
    dec.set_rate_match(E)
    out = dec.decode(llrE, want_info_llrs=False)
    for f in range(llrE.shape[0]):
        internal = subblock_deinterleave(derate_match_polar(llrE[f], 128), 128)
        n, c, m, il, b = oracle.decode_scl(internal, info, M, crc=POLY)
        assert out["n_paths"][f] == n
        np.testing.assert_array_equal(out["cands"][f, :n], c[:n])
        np.testing.assert_array_equal(out["metrics"][f, :n].view(np.int64), m[:n].view(np.int64))
        assert out["best_idx"][f] == b


def test_ties_golden_plain_kernels(golden):
    """The exact-tie golden cases (noiseless LLRs: equal metrics across paths) through the
    kernels without decision history, whose frozen re-ranks move paths between lanes and
    whose rankings take the tie key from the lane position (scl128_impl.h, kReorder)."""
    g = golden("g5_ties.npz")
    for key in map(str, g["keys"]):
        M = int(key.split("_M")[1])
        out = _native.get_decoder(128, g["info"], M, POLY).decode(g[key + "_llr"], want_info_llrs=False)
        n = g[key + "_npaths"]
        np.testing.assert_array_equal(out["n_paths"], n, err_msg=key)
        for f in range(len(n)):
            np.testing.assert_array_equal(out["cands"][f, :n[f]], g[key + "_cands"][f, :n[f]], err_msg=f"{key} f{f}")
            np.testing.assert_array_equal(out["metrics"][f, :n[f]], g[key + "_metrics"][f, :n[f]], err_msg=f"{key} f{f}")
        np.testing.assert_array_equal(out["best_idx"], g[key + "_best"], err_msg=key)


@pytest.mark.parametrize("M", [4, 8])
def test_quantized_llrs_plain_kernels_vs_oracle(M):
    """Integer-valued LLRs make exact metric ties common (equal increments in different orders);
    the plain kernels' lane-position tie keys and path moves against the oracle, bit for bit."""
    rng = np.random.default_rng(900 + M)
    info = construct_info_set(128, 64)
    B = 900
    llr = rng.integers(-4, 9, size=(B, 128)).astype(np.float64)
    llr[: B // 3] = rng.choice([-2.0, -1.0, 1.0, 2.0, 3.0], size=(B // 3, 128))
    out = _native.get_decoder(128, info, M, POLY).decode(llr, want_info_llrs=False)
    for f in range(B):
        n, c, m, il, b = oracle.decode_scl(llr[f], info, M, crc=POLY)
        assert out["n_paths"][f] == n, f
        np.testing.assert_array_equal(out["cands"][f, :n], c[:n], err_msg=f"M={M} f={f}")
        np.testing.assert_array_equal(out["metrics"][f, :n].view(np.int64), m[:n].view(np.int64))
        assert out["best_idx"][f] == b, f
