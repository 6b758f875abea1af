"""End-to-end FER parity on the GPU.

* run_fer_sweep --rng replay (the reference's own NumPy stream, HIP decoder) writes a CSV
  byte-identical to the reference's results/fer_M{8,4}.csv.
* DL-SCL retries (decode_with_retries and the batched form) match the reference's golden
  retry traces.
* --rng philox (on-device channel): FER within Monte-Carlo error of the reference.
"""
import math

import numpy as np
import pytest

from polar_code_amd.dlscl.flip import decode_with_retries, decode_with_retries_batch
from polar_code_amd.eval import run_fer_sweep

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [8, 4])
def test_cli_replay_reproduces_reference_csv(tmp_path, M):
    run_fer_sweep.main(["--M", str(M), "--frames", "2000", "--snr_lo", "5", "--snr_hi", "5", "--snr_step", "0",
                        "--retries", "8", "--beta", str(GOLDEN / f"beta_M{M}.npy"), "--seed", "0",
                        "--include_uncoded", "--out_dir", str(tmp_path), "--plot_dir", str(tmp_path), "--no_plot"])
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
