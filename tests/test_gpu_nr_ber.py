"""GPU: NR rate-matched decoding (front-end fused into the decode kernel) and the
run_ber_sweep CLI against the reference's golden rows."""
import numpy as np
import pytest

import oracle
from polar_code_amd.eval import run_ber_sweep as rb
from polar_code_amd.nr.polar import decode_rate_matched_scl, derate_match_polar, encode_rate_matched, \
    subblock_deinterleave
from polar_code_amd.polar.polar import construct_info_set
from polar_code_amd.utils.seeding import seed_all

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

CONFIGS = ["ber_polar_small", "ber_polar_128", "ber_dl_128", "ber_nr_256", "ber_nr_small"]


@pytest.mark.parametrize("name", CONFIGS)
def test_cli_rows_match_reference(golden, name, tmp_path):
    g = golden("g11_ber.npz")
    argv = [str(GOLDEN / "beta_M4.npy") if a == "BETA4" else a for a in str(g[name + "_argv"]).split()]
    out = tmp_path / "x.csv"
    rb.main(argv + ["--out", str(out)])
    assert out.read_text() == str(g[name])


def test_nr_decode_golden(golden):
    g = golden("g8_nr.npz")
    res = decode_rate_matched_scl(g["llrE"], "0x1864CFB", 128, 256, g["info"], 8)
    np.testing.assert_array_equal(res["best_path_bits"], g["bits"])
    np.testing.assert_array_equal(res["crc_pass"], g["crc_pass"])
    one = decode_rate_matched_scl(g["llrE"][0], "0x1864CFB", 128, 256, g["info"], 8)
    np.testing.assert_array_equal(one["payload"], g["bits"][0][:88])


@pytest.mark.parametrize("E", [100, 128, 200, 256, 300, 448])
def test_nr_fused_frontend_vs_host_frontend(E):
    rng = np.random.default_rng(E)
    info = construct_info_set(128, 88)
    llrE = rng.normal(2.0, 3.0, size=(64, E))
    res = decode_rate_matched_scl(llrE, "0x1864CFB", 128, E, info, 8)
    internal = np.stack([subblock_deinterleave(derate_match_polar(x, 128), 128) for x in llrE])
    bits, ok = oracle.decode_batch(internal, info, 8, "0x1864CFB")
    np.testing.assert_array_equal(res["best_path_bits"], bits)
    np.testing.assert_array_equal(res["crc_pass"], ok)


def test_nr_roundtrips():
    # reference tests/test_nr_polar.py:36-56, restated
    info = construct_info_set(128, 64)
    payload = np.random.default_rng(1).integers(0, 2, size=40, dtype=np.int8)
    tx = encode_rate_matched(payload, "0x1864CFB", 128, 128, info)
    res = decode_rate_matched_scl(np.where(tx == 0, 50.0, -50.0), "0x1864CFB", 128, 128, info, 4)
    assert res["crc_pass"]
    np.testing.assert_array_equal(res["payload"][:40], payload)
    seed_all(123)
    payload = np.random.randint(0, 2, size=40, dtype=np.int8)
    tx = encode_rate_matched(payload, "0x1864CFB", 128, 128, info)
    llr = 2.0 * ((1.0 - 2.0 * tx) + np.random.normal(0.0, 0.3, size=tx.shape)) / (0.3 ** 2)
    assert decode_rate_matched_scl(llr, "0x1864CFB", 128, 128, info, 4)["crc_pass"]


def test_nr_channel_kernel_roundtrip():
    """TX kernel with rate matching: at high SNR every frame decodes to its message."""
    from polar_code_amd import _native

    info = construct_info_set(128, 88)
    dec = _native.Decoder(128, info, 8, "0x1864CFB")
    dec.set_rate_match(256)
    B = 4096
    with _native.DeviceArena(dec) as mem:
        d_llr, d_msg = mem.alloc(B * 256 * 8), mem.alloc(B * 2 * 8)
        dec.channel_device(7, 1, 8.0, 64 / 256, 64, 0, B, d_llr, d_msg)
        llr = mem.download(d_llr, B * 256 * 8, np.float64).reshape(B, 256)
        msgw = mem.download(d_msg, B * 16, np.uint64).reshape(B, 2)
    out = dec.decode(llr, want_metrics=False, want_cands=False, want_info_llrs=False)
    msg = ((msgw[:, :, None] >> np.arange(64, dtype=np.uint64)) & 1).reshape(B, 128)[:, :88].astype(np.int8)
    assert out["crc_pass"].all()
    np.testing.assert_array_equal(out["best_bits"], msg)
