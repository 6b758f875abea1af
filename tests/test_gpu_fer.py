"""End-to-end FER parity on the GPU.

* run_fer_sweep --rng replay (the reference's own NumPy stream, HIP decoder) writes a CSV
  byte-identical to the reference's results/fer_M{8,4}.csv.
* DL-SCL retries (decode_with_retries, the host-ranked batch form and the on-device retry
  loop) match the reference's golden retry traces; the device loop equals the host-ranked
  form frame for frame on larger sets.
* --rng philox (on-device channel): FER within Monte-Carlo error of the reference.
"""
import math
from pathlib import Path

import numpy as np
import pytest

from polar_code_amd import _native
from polar_code_amd.dlscl.flip import decode_with_retries, decode_with_retries_batch, decode_with_retries_device
from polar_code_amd.eval import run_fer_sweep

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


# the run_fer_sweep invocations that produced the reference's committed results/fer_M{M}.csv
# (provenance recovered in SURVEY.md §6; M=1 pinned by the oracle, tests/test_replay_fer.py)
REF_RUNS = {
    8: ["--frames", "2000", "--snr_lo", "5", "--snr_hi", "5", "--snr_step", "0"],
    4: ["--frames", "2000", "--snr_lo", "5", "--snr_hi", "5", "--snr_step", "0"],
    1: ["--frames", "3000", "--snr_lo", "4.5", "--snr_hi", "6.0", "--snr_step", "0.5"],  # BASELINE config 1
}


@pytest.mark.parametrize("engine", ["device", "host"])
@pytest.mark.parametrize("M", [8, 4, 1])
def test_cli_replay_reproduces_reference_csv(tmp_path, M, engine):
    run_fer_sweep.main(["--M", str(M), *REF_RUNS[M], "--retries", "8", "--beta", str(GOLDEN / f"beta_M{M}.npy"),
                        "--seed", "0", "--include_uncoded", "--out_dir", str(tmp_path), "--plot_dir", str(tmp_path),
                        "--no_plot", "--dl_engine", engine])
    got = (tmp_path / f"fer_M{M}.csv").read_text()
    assert got == (GOLDEN / f"ref_fer_M{M}.csv").read_text()


def test_flip_retries_golden(golden):
    g = golden("g7_flip.npz")
    for tag, beta in (("beta", g["beta"]), ("none", None)):
        batch = decode_with_retries_batch(g["llr"], g["info"], 4, 8, crc="0x1864CFB", beta=beta)
        for f, llr in enumerate(g["llr"][:12]):
            r = decode_with_retries(llr, g["info"], 4, 8, crc="0x1864CFB", beta=beta)
            exp = [int(t) for t in g[f"{tag}_tried"][f] if t >= 0]
            assert r["tried_indices"] == exp
            assert len(r["attempts"]) == g[f"{tag}_attempts"][f]
            assert r["success"] == bool(g[f"{tag}_success"][f])
            np.testing.assert_array_equal(r["best_path_bits"], g[f"{tag}_bits"][f])
        np.testing.assert_array_equal(batch["best_bits"], g[f"{tag}_bits"])
        np.testing.assert_array_equal(batch["success"], g[f"{tag}_success"])
        np.testing.assert_array_equal(batch["attempts"], g[f"{tag}_attempts"])
        np.testing.assert_array_equal(batch["tried"], g[f"{tag}_tried"])


def test_device_retry_loop_golden(golden):
    g = golden("g7_flip.npz")
    for tag, beta in (("beta", g["beta"]), ("none", None)):
        out = decode_with_retries_device(g["llr"], g["info"], 4, 8, crc="0x1864CFB", beta=beta, msg=g["msg"])
        np.testing.assert_array_equal(out["best_bits"], g[f"{tag}_bits"])
        np.testing.assert_array_equal(out["success"], g[f"{tag}_success"])
        np.testing.assert_array_equal(out["attempts"], g[f"{tag}_attempts"])
        np.testing.assert_array_equal(out["tried"], g[f"{tag}_tried"])
        cd = out["counters"]["dl"]
        assert cd[0] == len(g["llr"]) and cd[1] == int((~g[f"{tag}_success"].astype(bool)).sum())
        assert cd[5] == int((g[f"{tag}_attempts"] - 1).sum())


# (1.5 dB: most frames fail, more than half of the chunk goes to one retry chain)
@pytest.mark.parametrize("M,retries,ebno,screen", [(4, 8, 3.0, "0"), (8, 8, 3.5, "0"), (2, 3, 3.0, "0"), (1, 70, 4.0, "0"),
                                                   (4, 8, 1.5, "0"), (4, 8, 2.0, "1"), (8, 8, 2.5, "1"),
                                                   (8, 8, 2.5, "2"), (4, 8, 2.0, "adaptive"), (8, 8, 3.5, "1"),
                                                   (4, 8, 3.0, "1"), (8, 8, 2.5, "1/2lane"), (4, 8, 2.0, "1/2lane"),
                                                   (4, 8, 3.0, "2"), (8, 8, 2.5, "1/fp"), (4, 8, 2.0, "1/fp"),
                                                   (8, 8, 3.5, "1/fp"), (4, 8, 3.0, "1/fp"), (8, 3, 1.5, "1/fp"),
                                                   (8, 8, 2.5, "1/nofp"), (4, 8, 2.0, "1/nofp")])
def test_device_retry_loop_equals_host_ranking(monkeypatch, M, retries, ebno, screen):
    """Device retry loop == numpy-ranked retries, frame by frame (3000 frames, ~30% failing);
    screen = 1: the retry decodes on the forced-bit screening instance (lane per path: per-frame
    forced / growing / full list) plus the exact decode of the entries it defers (tuning knob
    dl_screen = 1); "1/2lane": the same on the two-lanes-per-path instance (dl_retry_lane = 2);
    2: never (the exact forced-bit kernel); 0: the default (every chain screened where the list size
    has a screening instance, L = 4 and 8); "adaptive": the size-threshold rule with a threshold
    every chain here exceeds (dl_screen_min = 1); "1/fp" / "1/nofp": screened with the post pass
    fused into the retry decodes or the separate dl_post_kernel (dl_fused_post = 1 / 2)."""
    from polar_code_amd.polar.polar import construct_info_set, encode
    from polar_code_amd.polar.crc import attach_crc


    rng = np.random.default_rng(M * 100 + retries)
    info = construct_info_set(128, 64)
    msg = attach_crc(rng.integers(0, 2, size=(3000, 40), dtype=np.int8), "0x1864CFB")
    var = 1.0 / (2.0 * 0.5 * 10 ** (ebno / 10))
    llr = 2.0 * ((1.0 - 2.0 * encode(msg)) + rng.normal(0, math.sqrt(var), size=(3000, 128))) / var
    beta = np.load(GOLDEN / "beta_M4.npy")
    shared = _native.get_decoder(128, info, M, "0x1864CFB")  # (the handle the device loop uses)
    for b in (beta, None):
        p0 = shared.path_stats()
        dev = decode_with_retries_device(llr, info, M, retries, crc="0x1864CFB", beta=b,
                                         tuning=({"dl_screen": int(screen)} if screen.isdigit() else
                                                 {"dl_screen": 1, "dl_retry_lane": 2} if screen == "1/2lane" else
                                                 {"dl_screen": 1, "dl_fused_post": 1} if screen == "1/fp" else
                                                 {"dl_screen": 1, "dl_fused_post": 2} if screen == "1/nofp" else
                                                 {"dl_screen": 0, "dl_screen_min": 1}))
        p1 = shared.path_stats()
        if screen in ("1/fp", "1/nofp"):  # (the schedule under test ran)
            fused, sep = p1["fused_post_rounds"] - p0["fused_post_rounds"], p1["post_rounds"] - p0["post_rounds"]
            assert (fused > 0 and sep == 0) if screen == "1/fp" else (fused == 0 and sep > 0), (screen, fused, sep)
        host = decode_with_retries_batch(llr, info, M, retries, crc="0x1864CFB", beta=b)
        assert 0.05 < (~dev["base_pass"]).mean() < (0.97 if ebno < 2 else 0.9)
        np.testing.assert_array_equal(dev["tried"], host["tried"])
        np.testing.assert_array_equal(dev["attempts"], host["attempts"])
        np.testing.assert_array_equal(dev["best_bits"], host["best_bits"])
        np.testing.assert_array_equal(dev["success"], host["success"])


@pytest.mark.parametrize("K,M,ebno", [(100, 8, 3.0), (48, 16, 1.0)])
def test_device_retry_loop_runtime_info_set(K, M, ebno):
    """DL-SCL on an N = 128 code without a compiled-in kernel (its baseline screened by the runtime-
    information-set lane kernel; exact forced-bit retry decodes) equals the
    numpy-ranked retries frame for frame, beta = None (the checkpoints are K = 64)."""
    from polar_code_amd.polar.polar import construct_info_set
    from polar_code_amd.polar.crc import attach_crc

    rng = np.random.default_rng(K + M)
    info = construct_info_set(128, K)
    B = 2000
    msg = attach_crc(rng.integers(0, 2, size=(B, K - 24), dtype=np.int8), "0x1864CFB")
    u = np.zeros((B, 128), np.int8)
    u[:, info] = msg
    from polar_code_amd.polar.polar import _polar_transform
    var = 1.0 / (2.0 * K / 128 * 10 ** (ebno / 10))
    llr = 2.0 * ((1.0 - 2.0 * _polar_transform(u)) + rng.normal(0, math.sqrt(var), size=(B, 128))) / var
    dev = decode_with_retries_device(llr, info, M, 6, crc="0x1864CFB", beta=None)
    host = decode_with_retries_batch(llr, info, M, 6, crc="0x1864CFB", beta=None)
    assert 0.02 < (~dev["base_pass"]).mean() < 0.95
    for k in ("tried", "attempts", "best_bits", "success"):
        np.testing.assert_array_equal(dev[k], host[k], err_msg=k)


def test_philox_device_and_host_dl_engines_agree(tmp_path):
    rows = {}
    for engine in ("device", "host"):
        rows[engine] = run_fer_sweep.run_sweep(run_fer_sweep.build_argparser().parse_args(
            ["--M", "4", "--frames", "60000", "--snr_lo", "3.5", "--snr_hi", "4", "--snr_step", "0.5", "--retries",
             "8", "--beta", str(GOLDEN / "beta_M4.npy"), "--rng", "philox", "--batch", "30000", "--out_dir",
             str(tmp_path), "--plot_dir", str(tmp_path), "--no_plot", "--dl_engine", engine]))
    assert rows["device"] == rows["host"]
    assert rows["device"][0]["fer_dl"] < rows["device"][0]["fer_scl"]


def test_philox_fer_matches_reference_statistically(tmp_path):
    rows = run_fer_sweep.run_sweep(run_fer_sweep.build_argparser().parse_args(
        ["--M", "8", "--frames", "400000", "--snr_lo", "5", "--snr_hi", "5", "--snr_step", "0", "--retries", "8",
         "--beta", str(GOLDEN / "beta_M8.npy"), "--rng", "philox", "--batch", "200000", "--include_uncoded",
         "--out_dir", str(tmp_path), "--plot_dir", str(tmp_path), "--no_plot"]))
    r = rows[0]
    for key, ref_errs in (("fer_scl", 26), ("fer_dl", 20)):
        p_ref = ref_errs / 2000
        p = r[key]
        pp = (p * 400000 + ref_errs) / 402000
        z = (p - p_ref) / math.sqrt(pp * (1 - pp) * (1 / 400000 + 1 / 2000))
        assert abs(z) < 3, (key, p, p_ref, z)
    assert abs(r["fer_uncoded"] - 0.218) < 0.01


def test_config3_grid_sweep(tmp_path):
    """BASELINE config 3's shape: L=8, 6 SNR points 4.0-6.5 dB, DL-SCL with beta_M8.  The
    reference publishes only the 5 dB point (results/fer_M8.csv), so the other points are
    parity unpinned; they are held to the curve's shape: FER falls with SNR, DL-SCL never
    loses frames against its own SCL baseline, and 5 dB agrees with the reference (|z| < 3)."""
    rows = run_fer_sweep.run_sweep(run_fer_sweep.build_argparser().parse_args(
        ["--M", "8", "--frames", "200000", "--snr_lo", "4.0", "--snr_hi", "6.5", "--snr_step", "0.5", "--retries",
         "8", "--beta", str(GOLDEN / "beta_M8.npy"), "--rng", "philox", "--batch", "200000", "--out_dir",
         str(tmp_path), "--plot_dir", str(tmp_path), "--no_plot"]))
    assert [r["snr_db"] for r in rows] == [4.0, 4.5, 5.0, 5.5, 6.0, 6.5]
    scl = [r["fer_scl"] for r in rows]
    assert all(a > b for a, b in zip(scl, scl[1:])), scl
    assert all(r["fer_dl"] <= r["fer_scl"] for r in rows)
    p, p_ref = rows[2]["fer_scl"], 26 / 2000
    pp = (p * 200000 + 26) / 202000
    assert abs((p - p_ref) / math.sqrt(pp * (1 - pp) * (1 / 200000 + 1 / 2000))) < 3
    assert (tmp_path / "fer_M8.csv").exists()


def test_device_retry_loop_chunked_pipeline():
    """The chunked retry pipeline (retry rounds of chunk c overlapped with the baseline of c+1)
    gives the same per-frame results as the host ranking."""
    from polar_code_amd.polar.polar import construct_info_set, encode
    from polar_code_amd.polar.crc import attach_crc

    rng = np.random.default_rng(77)
    info = construct_info_set(128, 64)
    msg = attach_crc(rng.integers(0, 2, size=(5000, 40), dtype=np.int8), "0x1864CFB")
    var = 1.0 / (2.0 * 0.5 * 10 ** (3.0 / 10))
    llr = 2.0 * ((1.0 - 2.0 * encode(msg)) + rng.normal(0, math.sqrt(var), size=(5000, 128))) / var
    beta = np.load(GOLDEN / "beta_M4.npy")
    dev = decode_with_retries_device(llr, info, 4, 8, crc="0x1864CFB", beta=beta, msg=msg, tuning={"dl_chunks": 3})
    host = decode_with_retries_batch(llr, info, 4, 8, crc="0x1864CFB", beta=beta)
    np.testing.assert_array_equal(dev["tried"], host["tried"])
    np.testing.assert_array_equal(dev["attempts"], host["attempts"])
    np.testing.assert_array_equal(dev["best_bits"], host["best_bits"])
    assert dev["counters"]["dl"][1] == int((~host["success"]).sum())


@pytest.mark.parametrize("chunks,split", [("1", "2"), ("2", "2"), ("1", "1")])
def test_device_retry_loop_split_chains(chunks, split):
    """Two concurrent retry chains per chunk (each on its own stream, >= 4096 failing frames)
    give the same per-frame results as the host ranking."""
    from polar_code_amd.polar.polar import construct_info_set, encode
    from polar_code_amd.polar.crc import attach_crc

    rng = np.random.default_rng(78)
    B = 24000
    info = construct_info_set(128, 64)
    msg = attach_crc(rng.integers(0, 2, size=(B, 40), dtype=np.int8), "0x1864CFB")
    var = 1.0 / (2.0 * 0.5 * 10 ** (1.0 / 10))
    llr = 2.0 * ((1.0 - 2.0 * encode(msg)) + rng.normal(0, math.sqrt(var), size=(B, 128))) / var
    beta = np.load(GOLDEN / "beta_M4.npy")
    dev = decode_with_retries_device(llr, info, 4, 8, crc="0x1864CFB", beta=beta, msg=msg,
                                     tuning={"dl_chunks": int(chunks), "dl_split": int(split)})
    host = decode_with_retries_batch(llr, info, 4, 8, crc="0x1864CFB", beta=beta)
    assert (dev["attempts"] > 1).sum() >= 4096 * int(chunks) + 1000  # every chunk splits
    np.testing.assert_array_equal(dev["tried"], host["tried"])
    np.testing.assert_array_equal(dev["attempts"], host["attempts"])
    np.testing.assert_array_equal(dev["best_bits"], host["best_bits"])
    assert dev["counters"]["dl"][1] == int((~host["success"]).sum())


@pytest.mark.parametrize("L,depth,split,tune", [(4, 2, 0, {}), (8, 2, 0, {}), (4, 4, 0, {}), (8, 3, 0, {}), (4, 3, 2, {}),
                                                (4, 2, 0, {"post_epw": 4}), (8, 3, 0, {"post_epw": 4}),
                                                (4, 2, 0, {"post_epw": 2}), (4, 3, 0, {"dl_warm_apx": 1}),
                                                (8, 2, 0, {"dl_warm_apx": 2}), (4, 2, 0, {"dl_tail": 1}),
                                                (8, 4, 0, {"dl_tail": 1})])
def test_pipelined_dlscl_calls_equal_stream_ordered(L, depth, split, tune):
    """pscl_set_pipelined on pscl_dlscl_device: each call's retry chains and DL counters stay on
    the retry streams and overlap the next call's baseline (and, in the other chain set, the
    previous call's chains); split 0 = the pipelined default (one chain per call), 2 = two; tune:
    the narrow post pass's entries per wavefront (PSCL_TUNE_POST_EPW), screening-tail warm starts
    (PSCL_TUNE_DL_WARM_APX), the baseline tail on the handle's stream (PSCL_TUNE_DL_TAIL; by default
    it runs on a stream of its own beside the next call's baseline).  Calls on `depth` rotating output buffers (as bench.py's steps): a
    call's buffers are reused by the depth-th following call, which must start after that call's
    chains end.  After a join the last `depth` calls' bits, flags and attempts and the SCL/DL
    counters of all calls equal the stream-ordered calls'."""
    from polar_code_amd.polar.polar import construct_info_set

    info = construct_info_set(128, 64)
    beta = np.load(GOLDEN / f"beta_M{L}.npy")
    B, nb, nc = 40_000, depth + 3, _native.PSCL_NCOUNT
    res = {}
    for pipe in (True, False):
        dec = _native.Decoder(128, info, L, "0x1864CFB")
        dec.set_pipelined(pipe, depth=depth)
        if split:
            dec.set_tuning(dl_split=split)
        if tune:
            dec.set_tuning(**tune)
        with _native.DeviceArena(dec) as mem:
            d_llr = [mem.alloc(B * 128 * 8) for _ in range(nb)]
            d_msg = [mem.alloc(B * 8) for _ in range(nb)]
            d_out = [(mem.alloc(B * 8), mem.alloc(B), mem.alloc(B * 4)) for _ in range(depth)]
            d_cnt = mem.alloc(2 * nc * 8)
            mem.memset(d_cnt, 0, 2 * nc * 8)
            for i in range(nb):
                dec.channel_device(5, 60 + i, 2.5 + 0.5 * (i % 3), 0.5, 40, i * B, B, d_llr[i], d_msg[i])
            for i in range(nb):
                o = d_out[i % depth]
                dec.dlscl_device(d_llr[i], B, 8, beta=beta, d_best=o[0], d_flags=o[1], d_attempts=o[2],
                                 d_ref=d_msg[i], k_payload=40, d_counters_scl=d_cnt, d_counters_dl=d_cnt + nc * 8)
            dec.join()
            if "post_epw" in tune:
                assert (dec.path_stats()["post_epw4_launches"] > 0) == (pipe and tune["post_epw"] == 4)
            res[pipe] = ([(mem.download(b, B * 8, np.uint64), mem.download(f, B, np.uint8),
                           mem.download(a, B * 4, np.int32)) for b, f, a in d_out],
                         mem.download(d_cnt, 2 * nc * 8, np.int64).reshape(2, nc))
        dec.close()
    for i in range(depth):
        for k, name in enumerate(("best", "flags", "attempts")):
            np.testing.assert_array_equal(res[True][0][i][k], res[False][0][i][k], err_msg=f"{name}, buffer {i}")
    np.testing.assert_array_equal(res[True][1], res[False][1], err_msg="counters")
    c = res[True][1]
    assert c[0][0] == nb * B and c[1][1] <= c[0][1] and (res[True][0][0][2] > 1).sum() > 1000


@pytest.mark.parametrize("E_after", [0, 192])
def test_rate_match_switch_orders_pipelined_chains(E_after):
    """pscl_set_rate_match between a pipelined DL-SCL call on rate-matched rows ([B][E], E = 256,
    the (128, 88) NR code) and its join: the call's retry chains, still deferred, are enqueued
    with the E their rows were written for before the switch, so the outputs, attempts and
    counters equal the stream-ordered call's (the chains used to read the new E)."""
    from polar_code_amd.polar.polar import construct_info_set

    info = construct_info_set(128, 88)
    B, E, nc = 20_000, 256, _native.PSCL_NCOUNT
    res = {}
    for pipe in (True, False):
        dec = _native.Decoder(128, info, 4, "0x1864CFB")
        dec.set_pipelined(pipe)
        dec.set_rate_match(E)
        with _native.DeviceArena(dec) as mem:
            d_llr, d_msg = mem.alloc(B * E * 8), mem.alloc(B * 16)
            d_out = (mem.alloc(B * 16), mem.alloc(B), mem.alloc(B * 4))
            d_cnt = mem.alloc(2 * nc * 8)
            mem.memset(d_cnt, 0, 2 * nc * 8)
            dec.channel_device(3, 17, 1.5, 64.0 / E, 64, 0, B, d_llr, d_msg)
            dec.dlscl_device(d_llr, B, 8, d_best=d_out[0], d_flags=d_out[1], d_attempts=d_out[2], d_ref=d_msg,
                             k_payload=64, d_counters_scl=d_cnt, d_counters_dl=d_cnt + nc * 8)
            dec.set_rate_match(E_after)  # (the pipelined call's chains are still deferred here)
            dec.join()
            res[pipe] = [mem.download(d_out[0], B * 16, np.uint64), mem.download(d_out[1], B, np.uint8),
                         mem.download(d_out[2], B * 4, np.int32), mem.download(d_cnt, 2 * nc * 8, np.int64)]
        dec.close()
    for k, name in enumerate(("best", "flags", "attempts", "counters")):
        np.testing.assert_array_equal(res[True][k], res[False][k], err_msg=name)
    assert (res[True][2] > 1).sum() > 100  # retries ran


def test_device_free_orders_pipelined_chains():
    """pscl_device_free on the buffers of a pipelined DL-SCL call whose retry chains are still
    deferred (no join): the free first enqueues and completes those chains, so freeing the call's
    input rows and reference words right after it leaves its outputs and counters equal to the
    stream-ordered call's."""
    import ctypes as C

    from polar_code_amd.polar.polar import construct_info_set

    info = construct_info_set(128, 64)
    beta = np.load(GOLDEN / "beta_M4.npy")
    B, nc = 30_000, _native.PSCL_NCOUNT
    res = {}
    for pipe in (True, False):
        dec = _native.Decoder(128, info, 4, "0x1864CFB")
        dec.set_pipelined(pipe)
        with _native.DeviceArena(dec) as mem:
            d_out = (mem.alloc(B * 8), mem.alloc(B), mem.alloc(B * 4))
            d_cnt = mem.alloc(2 * nc * 8)
            mem.memset(d_cnt, 0, 2 * nc * 8)
            raw = []
            for nbytes in (B * 128 * 8, B * 8):
                p = C.c_void_p()
                _native.check(_native.lib().pscl_device_alloc(dec.handle, C.byref(p), nbytes))
                raw.append(p.value)
            d_llr, d_msg = raw
            dec.channel_device(9, 71, 2.5, 0.5, 40, 0, B, d_llr, d_msg)
            dec.dlscl_device(d_llr, B, 8, beta=beta, d_best=d_out[0], d_flags=d_out[1], d_attempts=d_out[2],
                             d_ref=d_msg, k_payload=40, d_counters_scl=d_cnt, d_counters_dl=d_cnt + nc * 8)
            for p in raw:  # no join: the chains of a pipelined call are still deferred here
                _native.check(_native.lib().pscl_device_free(dec.handle, p))
            res[pipe] = ([mem.download(d_out[0], B * 8, np.uint64), mem.download(d_out[1], B, np.uint8),
                          mem.download(d_out[2], B * 4, np.int32)], mem.download(d_cnt, 2 * nc * 8, np.int64))
        dec.close()
    for k in range(3):
        np.testing.assert_array_equal(res[True][0][k], res[False][0][k])
    np.testing.assert_array_equal(res[True][1], res[False][1])
    assert (res[True][0][2] > 1).sum() > 500


@pytest.mark.parametrize("N,K,E,L", [(128, 88, 256, 8), (256, 128, 0, 4)])
def test_pipelined_dlscl_rate_matched_and_long(N, K, E, L):
    """Pipelined DL-SCL calls on the NR (128,88) code rate matched to E = 256 (config 5's code)
    and on a long code (N = 256: HIST retry decodes, dense per-pass state on one chain): four
    calls on two alternating output buffers equal the stream-ordered calls (bits, flags,
    attempts of the last two calls; SCL/DL counters of all four)."""
    from polar_code_amd.polar.polar import construct_info_set

    info = construct_info_set(N, K)
    kp, n_in = K - 24, (E or N)
    B, nb, nc = 6000, 4, _native.PSCL_NCOUNT
    res = {}
    for pipe in (True, False):
        dec = _native.Decoder(N, info, L, "0x1864CFB")
        if E:
            dec.set_rate_match(E)
        dec.set_pipelined(pipe)
        with _native.DeviceArena(dec) as mem:
            d_llr = [mem.alloc(B * n_in * 8) for _ in range(nb)]
            d_msg = [mem.alloc(B * 16) for _ in range(nb)]
            d_out = [(mem.alloc(B * 16), mem.alloc(B), mem.alloc(B * 4)) for _ in range(2)]
            d_cnt = mem.alloc(2 * nc * 8)
            mem.memset(d_cnt, 0, 2 * nc * 8)
            rate = kp / E if E else K / N
            for i in range(nb):
                dec.channel_device(9, 70 + i, 1.0 + 0.5 * i, rate, kp, i * B, B, d_llr[i], d_msg[i])
            for i in range(nb):
                o = d_out[i & 1]
                dec.dlscl_device(d_llr[i], B, 8, d_best=o[0], d_flags=o[1], d_attempts=o[2], d_ref=d_msg[i],
                                 k_payload=kp, d_counters_scl=d_cnt, d_counters_dl=d_cnt + nc * 8)
            dec.join()
            res[pipe] = ([(mem.download(b, B * 16, np.uint64), mem.download(f, B, np.uint8),
                           mem.download(a, B * 4, np.int32)) for b, f, a in d_out],
                         mem.download(d_cnt, 2 * nc * 8, np.int64).reshape(2, nc))
        dec.close()
    for i in range(2):
        for k, name in enumerate(("best", "flags", "attempts")):
            np.testing.assert_array_equal(res[True][0][i][k], res[False][0][i][k], err_msg=f"{name}, buffer {i}")
    np.testing.assert_array_equal(res[True][1], res[False][1], err_msg="counters")
    c = res[True][1]
    assert c[0][0] == nb * B and c[1][5] > 100  # retries ran


def test_simulate_one_call_equals_separate_calls():
    """pscl_simulate (TX + uncoded + SCL + DL-SCL + counters in one call) equals the separate
    device calls over the same frames, and frame ranges add up exactly."""
    from polar_code_amd.polar.polar import construct_info_set

    info = construct_info_set(128, 64)
    dec = _native.Decoder(128, info, 4, "0x1864CFB")
    beta = np.load(Path(__file__).resolve().parent / "golden" / "beta_M4.npy")
    dec.set_beta(beta)
    B, seed, sid, snr = 6000, 11, 40, 4.0
    one = dec.simulate(seed, sid, snr, 0.5, 40, 0, B, 8, include_uncoded=True)
    parts = dec.simulate(seed, sid, snr, 0.5, 40, 0, 2500, 8, True) + dec.simulate(seed, sid, snr, 0.5, 40, 2500,
                                                                                   B - 2500, 8, True)
    np.testing.assert_array_equal(one, parts)
    nc = _native.PSCL_NCOUNT
    with _native.DeviceArena(dec) as mem:
        d_llr, d_msg = mem.alloc(B * 128 * 8), mem.alloc(B * 8)
        d_best, d_flags, d_cnt = mem.alloc(B * 8), mem.alloc(B), mem.alloc(3 * nc * 8)
        mem.memset(d_cnt, 0, 3 * nc * 8)
        dec.channel_device(seed, sid, snr, 0.5, 40, 0, B, d_llr, d_msg)
        dec.uncoded_device(seed, sid, snr, 40, 0, B, d_cnt + 2 * nc * 8)
        dec.dlscl_device(d_llr, B, 8, beta=beta, d_best=d_best, d_flags=d_flags, d_ref=d_msg, k_payload=40,
                         d_counters_scl=d_cnt, d_counters_dl=d_cnt + nc * 8)
        sep = mem.download(d_cnt, 3 * nc * 8, np.int64).reshape(3, nc)
    np.testing.assert_array_equal(one, sep)
    assert one[0][0] == B and one[1][1] <= one[0][1] and one[2][0] == B


def test_pipelined_sweep_equals_per_point_simulate():
    """run_fer_sweep --rng philox enqueues the whole sweep on a pipelined handle
    (pscl_simulate_device: each block's DL-SCL chains overlap the next block's and the next SNR
    point's TX and baseline): every point's SCL, DL-SCL and uncoded counters equal the
    stream-ordered per-block pscl_simulate calls'."""
    from polar_code_amd.eval import run_fer_sweep as rfs
    from polar_code_amd.polar.polar import construct_info_set
    from polar_code_amd.utils.seeding import philox_stream_id

    info = construct_info_set(128, 64)
    beta = np.load(GOLDEN / "beta_M8.npy")
    args = rfs.build_argparser().parse_args(["--M", "8", "--retries", "8", "--rng", "philox", "--include_uncoded",
                                             "--batch", "70000", "--seed", "3"])
    pts = [3.5, 4.0, 5.0]
    ranges = [(0, 150_000), (20_000, 160_000), (0, 90_001)]
    got = rfs._philox_sweep_device(args, pts, ranges, info, beta, 0, 40)
    dec = _native.Decoder(128, info, 8, "0x1864CFB")
    dec.set_beta(beta)
    for i, (snr, (a, b)) in enumerate(zip(pts, ranges)):
        want = np.zeros((3, _native.PSCL_NCOUNT), np.int64)
        for b0 in range(a, b, 70000):
            want += dec.simulate(3, philox_stream_id(snr), snr, 0.5, 40, b0, min(b, b0 + 70000) - b0, 8, True)
        np.testing.assert_array_equal(got[i], want, err_msg=f"{snr} dB")
        assert want[1][_native.CNT_FRAME_ERR] <= want[0][_native.CNT_FRAME_ERR]
