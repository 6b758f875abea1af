"""GPU: BASELINE.json configs 2, 4 and 5 at their stated size (10^6-frame batches), every frame
checked against the oracle (C restatement of the reference, test infrastructure only).

Each test generates one 10^6-frame batch on the device with the Philox TX chain
(pscl_channel_device: payload -> CRC-24 -> polar encode [-> NR interleave/repeat] -> BPSK ->
AWGN -> LLR), decodes it through the C ABI exactly as bench.py and the sweeps do, copies the
LLRs back and decodes the same frames with the oracle.  Compared frame by frame: best bits,
CRC flag and (plain SCL) best candidate index, DL-SCL attempt counts; and the device-side
FER/BER counters against counts recomputed on the host from the decoded bits.

  config 2  SCL L=4 P(128,64)+CRC24, 10^6 frames at 5 dB        (scl.py:108-209)
  config 4  DL-SCL L=4, 8 flip retries, beta_M4, 10^6 frames     (flip.py:65-141)
  config 5  NR (128,88) rate matched to E=256, SCL L=8, 10^6      (scl_nr.py:40-57 front end)
Configs 1 and 3 are covered by test_gpu_fer.py (config 1's CSV byte-identical to the
reference's results/fer_M1.csv, config 3's 4.0-6.5 dB grid); config 3's DL-SCL decode (L = 8,
beta_M8) is checked here against the oracle at 4.0 and 4.5 dB, and config 4 with every retry
decode screened.
"""
import numpy as np
import pytest

import oracle
from conftest import GOLDEN
from polar_code_amd import _native
from polar_code_amd.dlscl.flip import words_to_bits
from polar_code_amd.nr.polar import derate_match_polar, subblock_deinterleave
from polar_code_amd.polar.polar import construct_info_set

pytestmark = pytest.mark.gpu
POLY = "0x1864CFB"
B = 1_000_000
EBNO = 5.0
FRAMES, FRAME_ERR, BIT_ERR, PAY_ERR, PAY_BIT, RETRIES = 0, 1, 2, 3, 4, 5


def _nr_internal(llrE: np.ndarray, N: int) -> np.ndarray:
    """Vectorised scl_nr.py:47-48 front end (derate_match_polar then subblock_deinterleave) for
    E = 2N; held to the package's per-frame mirrors on the first rows by the caller."""
    E = llrE.shape[1]
    assert E == 2 * N
    avg = (llrE[:, :N] + llrE[:, N:]) / 2.0  # two repeats summed in order, divided by the count
    nb = N // 32
    i = np.arange(N)
    order = (i % 32) * nb + i // 32
    out = np.empty_like(avg)
    out[:, order] = avg
    return out


def _batch(dec, mem, L, K, kp, E, seed):
    n_in = E or 128
    rate = kp / E if E else K / 128
    d_llr = mem.alloc(B * n_in * 8)
    d_msg = mem.alloc(B * dec.W * 8)
    dec.channel_device(seed, int(EBNO * 10), EBNO, rate, kp, 0, B, d_llr, d_msg)
    return d_llr, d_msg


def _host_counts(bits, msg_bits, ok, kp):
    err = bits != msg_bits
    return {FRAMES: bits.shape[0], FRAME_ERR: int(np.count_nonzero(~ok)), BIT_ERR: int(err.sum()),
            PAY_ERR: int(np.count_nonzero(err[:, :kp].any(axis=1))), PAY_BIT: int(err[:, :kp].sum())}


def _check_counters(cnt, host, tag):
    for k, v in host.items():
        assert int(cnt[k]) == v, f"{tag}: counter {k} device {int(cnt[k])} host {v}"


def _plain_config(L, E, seed):
    K = 88 if E else 64
    kp = K - 24
    info = construct_info_set(128, K)
    dec = _native.Decoder(128, info, L, POLY)
    if E:
        dec.set_rate_match(E)
    with _native.DeviceArena(dec) as mem:
        d_llr, d_msg = _batch(dec, mem, L, K, kp, E, seed)
        d_best, d_flags, d_cnt = mem.alloc(B * dec.W * 8), mem.alloc(B), mem.alloc(8 * 8)
        mem.memset(d_cnt, 0, 64)
        dec.decode_device(d_llr, B, d_best=d_best, d_flags=d_flags, d_ref=d_msg, k_payload=kp, d_counters=d_cnt)
        dec.sync()
        scr = dec.screening_count()
        best = mem.download(d_best, B * dec.W * 8, np.uint64).reshape(B, dec.W)
        flags = mem.download(d_flags, B, np.uint8)
        cnt = mem.download(d_cnt, 64, np.int64)
        msg = mem.download(d_msg, B * dec.W * 8, np.uint64).reshape(B, dec.W)
        llr = mem.download(d_llr, B * (E or 128) * 8, np.float64).reshape(B, E or 128)
    dec.close()
    if E:
        head = np.stack([subblock_deinterleave(derate_match_polar(r, 128), 128) for r in llr[:2000]])
        llr = _nr_internal(llr, 128)
        np.testing.assert_array_equal(llr[:2000], head)  # vectorised front end == the mirrors
    bits_o, ok_o, idx_o = oracle.decode_batch(llr, info, L, POLY, want_idx=True)
    bits = words_to_bits(best, K)
    ok = (flags & 0x80) != 0
    tag = f"L={L} E={E}"
    bad_bits = np.flatnonzero(np.any(bits != bits_o, axis=1))
    assert bad_bits.size == 0, f"{tag}: best bits differ from the oracle in {bad_bits.size} frames, first {bad_bits[:5]}"
    np.testing.assert_array_equal(ok, ok_o, err_msg=f"{tag}: CRC flags")
    np.testing.assert_array_equal((flags & 0x3F).astype(np.int32), idx_o, err_msg=f"{tag}: best index")
    _check_counters(cnt, _host_counts(bits, words_to_bits(msg, K), ok, kp), tag)
    return cnt, scr


def test_config2_scl_L4_1e6_frames_vs_oracle():
    cnt, scr = _plain_config(4, 0, seed=20)
    fer = cnt[FRAME_ERR] / cnt[FRAMES]
    # reference results/fer_M4.csv:2: 91/2000 frame errors at 5 dB; z within MC error
    p0 = 91 / 2000
    assert abs(fer - p0) < 4 * np.sqrt(p0 * (1 - p0) / 2000), fer
    assert 0 < scr < B // 20  # the screening pass ran and deferred a few frames to the exact kernel
    print(f"config 2: FER {fer:.5f}, {scr} frames re-decoded exactly, 0/{B} oracle mismatches")


def test_config5_nr_E256_L8_1e6_frames_vs_oracle():
    cnt, scr = _plain_config(8, 256, seed=50)
    assert cnt[FRAMES] == B and 0 < scr < B // 20
    print(f"config 5: payload FER {cnt[PAY_ERR] / B:.6f}, BER {cnt[PAY_BIT] / (B * 64):.3e}, 0/{B} oracle mismatches")


def _dl_config(L, beta_name, ebno, nb, seed, tuning=None, pipelined=False):
    """One DL-SCL batch of nb frames (8 flips, beta_<beta_name>) against the oracle's
    decode_with_retries, frame by frame; returns (SCL counters, DL counters, oracle attempts).
    pipelined: the call as bench.py's steps enqueue it (pscl_set_pipelined: the post pass's narrow
    form, PSCL_TUNE_POST_EPW)."""
    K, kp, R = 64, 40, 8
    info = construct_info_set(128, K)
    beta = np.load(GOLDEN / f"beta_{beta_name}.npy")
    dec = _native.Decoder(128, info, L, POLY)
    if tuning:
        dec.set_tuning(**tuning)
    if pipelined:
        dec.set_pipelined(True)
    with _native.DeviceArena(dec) as mem:
        d_llr, d_msg = mem.alloc(nb * 128 * 8), mem.alloc(nb * 8)
        dec.channel_device(seed, int(ebno * 10), ebno, K / 128, kp, 0, nb, d_llr, d_msg)
        d_best, d_flags, d_att = mem.alloc(nb * 8), mem.alloc(nb), mem.alloc(nb * 4)
        d_cs, d_cd = mem.alloc(64), mem.alloc(64)
        mem.memset(d_cs, 0, 64)
        mem.memset(d_cd, 0, 64)
        dec.dlscl_device(d_llr, nb, R, beta=beta, d_best=d_best, d_flags=d_flags, d_attempts=d_att, d_ref=d_msg,
                         k_payload=kp, d_counters_scl=d_cs, d_counters_dl=d_cd)
        if pipelined:
            dec.join()
        dec.sync()
        paths = dec.path_stats()
        if tuning and "lane_exact" in tuning:  # (exact retry rounds / side chain on the lane instance)
            assert (paths["lane_exact_launches"] > 0) == (tuning["lane_exact"] == 1), paths
        if tuning and "post_epw" in tuning:
            assert (paths["post_epw4_launches"] > 0) == (pipelined and tuning["post_epw"] == 4), paths
        if tuning and tuning.get("dl_fused_post") == 1:  # (the schedule under test ran)
            assert paths["fused_post_rounds"] > 0 and paths["post_rounds"] == 0, paths
        if tuning and tuning.get("dl_fused_post") == 2:
            assert paths["fused_post_rounds"] == 0 and paths["post_rounds"] > 0, paths
        best = mem.download(d_best, nb * 8, np.uint64).reshape(nb, 1)
        flags = mem.download(d_flags, nb, np.uint8)
        att = mem.download(d_att, nb * 4, np.int32)
        cs, cd = mem.download(d_cs, 64, np.int64), mem.download(d_cd, 64, np.int64)
        msg = mem.download(d_msg, nb * 8, np.uint64).reshape(nb, 1)
        llr = mem.download(d_llr, nb * 128 * 8, np.float64).reshape(nb, 128)
    dec.close()
    bits_o, ok_o, att_o = oracle.dl_batch(llr, info, L, R, POLY, beta)
    bits = words_to_bits(best, K)
    ok = (flags & 0x80) != 0
    bad = np.flatnonzero(np.any(bits != bits_o, axis=1) | (ok != ok_o) | (att != att_o))
    assert bad.size == 0, f"DL-SCL L={L} differs from the oracle in {bad.size} frames, first {bad[:5]}"
    _check_counters(cd, _host_counts(bits, words_to_bits(msg, K), ok, kp), "DL-SCL")
    assert int(cd[RETRIES]) == int((att_o - 1).sum())  # one re-decode per flip tried
    base_fail = int(cs[FRAME_ERR])
    assert cs[FRAMES] == nb and base_fail == int(np.count_nonzero(att_o > 1))  # retried iff the baseline failed
    return cs, cd, att_o


def test_config4_dlscl_L4_r8_beta4_1e6_frames_vs_oracle():
    cs, cd, _ = _dl_config(4, "M4", EBNO, B, seed=40)
    base_fail = int(cs[FRAME_ERR])
    # reference results/fer_M4.csv:2: SCL 91/2000, DL-SCL 71/2000 at 5 dB
    for got, ref in ((base_fail / B, 91 / 2000), (cd[FRAME_ERR] / B, 71 / 2000)):
        assert abs(got - ref) < 4 * np.sqrt(ref * (1 - ref) / 2000), (got, ref)
    print(f"config 4: SCL FER {base_fail / B:.5f}, DL-SCL FER {cd[FRAME_ERR] / B:.5f}, "
          f"{cd[RETRIES] / B:.3f} re-decodes/frame, 0/{B} oracle mismatches")


@pytest.mark.parametrize("L,beta,ebno,nb,tuning", [
    (8, "M8", 4.5, 200_000, {"dl_screen": 1}),   # config 3's DL-SCL point (L = 8: lane-per-path FS retry decodes)
    (8, "M8", 4.0, 100_000, {"dl_screen": 1, "dl_retry_lane": 2}),  # the two-lanes-per-path screening instance
    (4, "M4", 5.0, 1_000_000, {"dl_screen": 1}),  # config 4 with every retry decode screened (L = 4 lane FS)
    (8, "M8", 4.5, 200_000, {"dl_screen": 1, "dl_fused_post": 1}),  # the post pass fused into the retry decodes
    (4, "M4", 5.0, 1_000_000, {"dl_screen": 1, "dl_fused_post": 1}),
    (8, "M8", 4.5, 200_000, {"dl_screen": 1, "dl_fused_post": 2}),  # the separate post pass
    (8, "M8", 4.0, 200_000, {"dl_screen": 2, "lane_exact": 1}),  # every retry round exact, lane-per-path
    (4, "M4", 5.0, 1_000_000, {"dl_screen": 2, "lane_exact": 1}),
    (8, "M8", 4.0, 200_000, {"dl_screen": 2, "lane_exact": 2}),  # every retry round on the exact kernel
    (8, "M8", 4.5, 200_000, {"dl_screen": 1, "lane_exact": 2}),  # the side chain on the exact kernel
    (8, "M8", 4.5, 200_000, {"dl_screen": 1, "dl_warm_apx": 1}),  # screening-tail warm starts (default)
    (8, "M8", 4.5, 200_000, {"dl_screen": 1, "dl_warm_apx": 2}),  # exact warm starts, deferrals at their bucket
    (8, "M8", 4.0, 100_000, {"dl_screen": 1, "dl_warm_apx": 1, "dl_retry_lane": 2}),  # (two-lanes-per-path screening)
])
def test_dlscl_screened_retry_decodes_vs_oracle(L, beta, ebno, nb, tuning):
    """Screened DL-SCL retry rounds (forced-bit screening decodes + exact decodes of the entries
    they defer) against the oracle on every frame: bits, CRC flags, attempt counts, counters."""
    _screened_vs_oracle(L, beta, ebno, nb, tuning, False)


@pytest.mark.parametrize("L,beta,ebno,nb,tuning", [
    (4, "M4", 5.0, 1_000_000, {"post_epw": 4}),  # config 4 as the bench runs it: the narrow post pass, 4 entries per wavefront
    (8, "M8", 4.0, 200_000, {"post_epw": 4}),
    (8, "M8", 4.0, 200_000, {"post_epw": 2}),    # 2 entries per wavefront
    (4, "M4", 5.0, 1_000_000, {"dl_warm_apx": 1}),  # screening-tail warm starts, deferrals exact from phase 0
    (8, "M8", 4.0, 200_000, {"dl_warm_apx": 1}),
])
def test_dlscl_pipelined_post_forms_vs_oracle(L, beta, ebno, nb, tuning):
    """The narrow (pipelined) post pass in both forms (PSCL_TUNE_POST_EPW: 32 or 16 lanes per entry)
    and with screening-tail warm-start metrics (PSCL_TUNE_DL_WARM_APX) against the oracle on every
    frame."""
    _screened_vs_oracle(L, beta, ebno, nb, tuning, True)


def test_post_epw_knob_validated():
    dec = _native.Decoder(128, construct_info_set(128, 64), 4, POLY)
    for bad in (1, 3, 5):
        with pytest.raises(Exception):
            dec.set_tuning(post_epw=bad)
    dec.set_tuning(post_epw=4)
    dec.set_tuning(post_epw=0)
    dec.close()


def _screened_vs_oracle(L, beta, ebno, nb, tuning, pipelined):
    cs, cd, att_o = _dl_config(L, beta, ebno, nb, seed=60 + L, tuning=tuning, pipelined=pipelined)
    assert int(np.count_nonzero(att_o > 2)) > nb // 200  # many multi-round entries (warm starts, growth)
    print(f"L={L} {ebno} dB {tuning}: SCL FER {cs[FRAME_ERR] / nb:.5f}, DL-SCL FER {cd[FRAME_ERR] / nb:.5f}, "
          f"0/{nb} oracle mismatches")
