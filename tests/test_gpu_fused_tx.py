"""GPU: the fused TX (PSCL_TUNE_TX_FUSED) equals the separate TX launch bit for bit.

pscl_simulate[_device] runs one SNR point of run_fer_sweep's Monte-Carlo loop
(/root/reference/dl_scl_polar/eval/run_fer_sweep.py:79-121: payload -> CRC -> encode -> BPSK/AWGN ->
SCL + DL-SCL retries -> counts, plus the uncoded baseline).  With the TX chain fused, the baseline
decode (scl_lane_kernel TXF) draws each frame's channel row from channel_kernel's Philox stream
itself instead of reading it, and tx_rows_kernel writes only the rows of the frames the exact
re-decode (deferred) and the retry chain (CRC failing) read again.  Every counter -- SCL and DL-SCL
frame/bit/payload errors, retry decodes, the uncoded baseline's errors -- must equal the unfused
path's, at low SNR (many failing frames, many deferred ones) and at the BASELINE points."""
import numpy as np
import pytest

from polar_code_amd import _native
from polar_code_amd.polar.polar import construct_info_set
from polar_code_amd.utils.seeding import philox_stream_id

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
POLY = "0x1864CFB"


def _decoder(L, fused, beta):
    dec = _native.Decoder(128, construct_info_set(128, 64), L, POLY)
    dec.set_tuning(tx_fused=1 if fused else 2)
    dec.set_beta(beta)
    return dec


@pytest.mark.parametrize("L,ebno", [(8, 5.0), (8, 3.0), (8, 6.5), (4, 5.0), (4, 2.5)])
def test_fused_tx_simulate_equals_unfused(L, ebno):
    beta = np.load(GOLDEN / f"beta_M{L}.npy")
    B = 120_000
    out = {}
    for fused in (True, False):
        dec = _decoder(L, fused, beta)
        out[fused] = dec.simulate(0, philox_stream_id(ebno), ebno, 0.5, 40, 7_777, B, 8, include_uncoded=True)
        assert (dec.path_stats()["fused_tx_blocks"] > 0) == fused  # (the schedule under test ran)
        dec.close()
    np.testing.assert_array_equal(out[True], out[False])
    c = out[True]
    assert c[0][0] == B and c[2][0] == B  # SCL and uncoded frame counts
    assert c[0][1] > 0 and c[2][1] > 0     # errors on both (so the comparison bites)
    if ebno <= 3.0:
        assert c[1][5] > 1000              # retry decodes read the rows tx_rows_kernel wrote


@pytest.mark.parametrize("L", [8, 4])
def test_fused_tx_pipelined_sweep_equals_unfused(L):
    """A pipelined sweep of pscl_simulate_device calls (as run_fer_sweep --rng philox enqueues it:
    the retry chains of one point overlap the next point's TX and baseline) with the counters
    accumulated on the device: fused and unfused equal per point."""
    beta = np.load(GOLDEN / f"beta_M{L}.npy")
    B, pts, nc = 100_000, [4.0, 4.5, 5.0, 5.5], _native.PSCL_NCOUNT
    res = {}
    for fused in (True, False):
        dec = _decoder(L, fused, beta)
        dec.set_pipelined(True)
        with _native.DeviceArena(dec) as mem:
            d_cnt = [mem.alloc(3 * nc * 8) for _ in pts]
            for d in d_cnt:
                mem.memset(d, 0, 3 * nc * 8)
            for x, d in zip(pts, d_cnt):
                dec.simulate_device(0, philox_stream_id(x), x, 0.5, 40, 0, B, 8, True, d)
            dec.join()
            dec.sync()
            assert (dec.path_stats()["fused_tx_blocks"] >= len(pts)) == fused
            res[fused] = [mem.download(d, 3 * nc * 8, np.int64).reshape(3, nc) for d in d_cnt]
        dec.close()
    for i, x in enumerate(pts):
        np.testing.assert_array_equal(res[True][i], res[False][i], err_msg=f"{x} dB")


def test_fused_tx_knob_validated():
    dec = _native.Decoder(128, construct_info_set(128, 64), 8, POLY)
    with pytest.raises(Exception):
        dec.set_tuning(tx_fused=3)
    dec.close()
