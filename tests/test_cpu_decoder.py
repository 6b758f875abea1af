"""The product's host decoder (pscl_decode_cpu, csrc/scl_cpu.cpp) on a GPU-less host.

BASELINE config 1 runs run_fer_sweep on CPU, as the reference does (run_fer_sweep.py:41-191).
The product's CPU path is its own C++ decoder in libpolar_mi355x.so -- never oracle/ -- held
here to the reference's golden decode_scl outputs (every candidate, metric bit pattern and
decision LLR) and, through `run_fer_sweep --device cpu`, to the reference's committed
results/fer_M1.csv byte for byte.  No test here touches a GPU.
"""
import re
from pathlib import Path

import numpy as np
import pytest

from polar_code_amd import _native
from polar_code_amd.polar.scl import decode_scl

from conftest import GOLDEN, ROOT

DECODE_SETS = ["g4_decode.npz", "g6_forced.npz", "g10_n16.npz", "g10_n32.npz", "g10_n64_nocrc.npz",
               "g10_k88.npz", "g10_m16.npz", "g10_n8.npz", "g10_n4.npz", "g10_n2.npz",
               "g14_n256.npz", "g14_n256_forced.npz", "g14_n512.npz", "g14_n1024.npz"]


def _check_set(g, key, M, crc):
    llr = g[key + "_llr"]
    B, N = llr.shape
    force = g[key + "_force"] if key + "_force" in g.files else None
    dec = _native.CpuDecoder(N, g["info"], M, crc, threads=2)
    out = dec.decode(llr, force)
    for f in range(B):
        n = int(g[key + "_npaths"][f])
        assert out["n_paths"][f] == n, (key, f)
        np.testing.assert_array_equal(out["cands"][f, :n], g[key + "_cands"][f][:n], err_msg=f"{key} frame {f}")
        np.testing.assert_array_equal(out["metrics"][f, :n].view(np.int64),
                                      np.asarray(g[key + "_metrics"][f][:n], np.float64).view(np.int64),
                                      err_msg=f"{key} frame {f}")
        np.testing.assert_array_equal(out["info_llrs"][f, :n].view(np.int64),
                                      np.asarray(g[key + "_info_llrs"][f][:n], np.float64).view(np.int64),
                                      err_msg=f"{key} frame {f}")
        assert out["best_idx"][f] == g[key + "_best"][f], (key, f)
        np.testing.assert_array_equal(out["best_bits"][f], g[key + "_cands"][f][int(g[key + "_best"][f])])


@pytest.mark.parametrize("name", DECODE_SETS)
def test_cpu_decoder_reference_goldens(golden, name):
    g = golden(name)
    crc = str(g["crc"]) or None
    for key in g["keys"]:
        key = str(key)
        _check_set(g, key, int(key.split("_")[0][1:]), crc)


def test_cpu_decoder_reference_ties(golden):
    """Exact metric ties (noiseless and integer LLRs): python's stable sort order, bit for bit."""
    g = golden("g5_ties.npz")
    for key in g["keys"]:
        key = str(key)
        _check_set(g, key, int(key.split("_M")[1]), "0x1864CFB")


def test_decode_scl_device_cpu_and_errors(golden):
    """decode_scl(..., device="cpu") returns the reference's dict; the reference's argument
    errors map to the same exception types."""
    g = golden("g4_decode.npz")
    key = str(g["keys"][0])
    M = int(key.split("_")[0][1:])
    r = decode_scl(g[key + "_llr"][0], g["info"], M, crc="0x1864CFB", device="cpu")
    b = int(g[key + "_best"][0])
    np.testing.assert_array_equal(r["best_path_bits"], g[key + "_cands"][0][b])
    assert len(r["candidates"]) == int(g[key + "_npaths"][0])
    with pytest.raises(ValueError):
        _native.CpuDecoder(96, g["info"], 4, "0x1864CFB")
    with pytest.raises(ValueError):
        _native.CpuDecoder(128, np.arange(10), 4, "0x1864CFB")  # message shorter than the CRC
    dec = _native.CpuDecoder(128, g["info"], 4, "0x1864CFB")
    with pytest.raises(ValueError):
        dec.decode(g[key + "_llr"][:1], np.full((1, g["info"].size), 2, np.int8))


def test_run_fer_sweep_device_cpu_reproduces_reference_m1_csv(tmp_path):
    """BASELINE config 1 on the CPU: `run_fer_sweep --M 1 --device cpu` (SC = SCL M=1, DL-SCL with
    8 flips and beta_M1, uncoded baseline, the reference's seed-0 NumPy stream) writes the
    reference's results/fer_M1.csv (3000 frames per point, 4.5-6.0 dB) byte for byte."""
    from polar_code_amd.eval import run_fer_sweep as rfs

    args = rfs.build_argparser().parse_args(
        ["--M", "1", "--frames", "3000", "--snr_lo", "4.5", "--snr_hi", "6.0", "--snr_step", "0.5", "--retries", "8",
         "--beta", str(GOLDEN / "beta_M1.npy"), "--seed", "0", "--include_uncoded", "--device", "cpu",
         "--out_dir", str(tmp_path), "--plot_dir", str(tmp_path), "--no_plot"])
    rfs.run_sweep(args)
    assert (tmp_path / "fer_M1.csv").read_text() == (GOLDEN / "ref_fer_M1.csv").read_text()


def test_product_package_never_imports_the_oracle():
    """The product (polar_code_amd/) has no code path into oracle/: no import of it anywhere."""
    pat = re.compile(r"^\s*(from\s+oracle\b|import\s+oracle\b|from\s+\.+oracle\b)|oracle\.(decode|dl_batch|run)",
                     re.M)
    hits = [str(p) for p in (ROOT / "polar_code_amd").rglob("*.py") if pat.search(p.read_text())]
    assert hits == []
