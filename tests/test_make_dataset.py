"""make_dataset (polar_code_amd/train/make_dataset.py) against the reference's shards.

tests/golden/g12_dataset.npz holds the reference's generate_samples output for two small
low-SNR runs (make_golden.py g12).  CPU: the host logic (replayed NumPy stream, failing-frame
selection, float32 |L0| argsort order, flip schedule, labels, meta) with the C oracle as the
decoder.  GPU: the shipped path (batched GPU decodes + decision-LLR replay), same shards.
"""
import json

import numpy as np
import pytest

import oracle
from polar_code_amd.train import make_dataset as md

from conftest import GOLDEN

CONFIGS = ["m4_2p5db", "m8_3db"]


def _oracle_decode_batch(llr, info_set, M, crc, forced=None):
    info = np.asarray(info_set, np.int32)
    bits = np.zeros((llr.shape[0], info.size), np.int8)
    ok = np.zeros(llr.shape[0], bool)
    for b in range(llr.shape[0]):
        n, c, m, il, best = oracle.decode_scl(llr[b], info, M, crc, None if forced is None else forced[b])
        bits[b] = c[best]
        ok[b] = oracle.check_crc(bits[b], crc)
    return bits, ok


def _oracle_best_path_llrs(llr, info_set, M, crc, bits):
    info = np.asarray(info_set, np.int32)
    out = np.zeros((llr.shape[0], info.size))
    for b in range(llr.shape[0]):
        n, c, m, il, best = oracle.decode_scl(llr[b], info, M, crc)
        assert np.array_equal(c[best], bits[b])
        out[b] = il[best]
    return out


def _check(tmp_path, name):
    g = np.load(GOLDEN / "g12_dataset.npz")
    argv = str(g[name + "_argv"]).split()
    shard = md.generate_samples(md.build_argparser().parse_args(argv + ["--out", str(tmp_path / "ds"),
                                                                       "--batch", "128"]))
    z = np.load(shard)
    np.testing.assert_array_equal(z["abs_l0"], g[name + "_abs_l0"])
    np.testing.assert_array_equal(z["flip_idx"], g[name + "_flip_idx"])
    assert json.loads(str(z["meta"])) == json.loads(str(g[name + "_meta"]))


@pytest.mark.parametrize("name", CONFIGS)
def test_dataset_host_logic_with_oracle(tmp_path, monkeypatch, name):
    monkeypatch.setattr(md, "decode_batch", _oracle_decode_batch)
    monkeypatch.setattr(md, "best_path_llrs", _oracle_best_path_llrs)
    _check(tmp_path, name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CONFIGS)
def test_dataset_gpu_matches_reference(tmp_path, name):
    _check(tmp_path, name)


@pytest.mark.gpu
def test_dataset_philox_mode(tmp_path):
    shard = md.generate_samples(md.build_argparser().parse_args(
        ["--M", "4", "--snr_db", "2.5", "--frames", "20000", "--out", str(tmp_path / "p"), "--rng", "philox",
         "--batch", "8192"]))
    z = np.load(shard)
    meta = json.loads(str(z["meta"]))
    assert z["abs_l0"].shape == (meta["samples"], 64) and z["abs_l0"].dtype == np.float32
    assert z["flip_idx"].dtype == np.int32 and (z["flip_idx"] >= 0).all() and (z["flip_idx"] < 64).all()
    # reference run at the same point: 79 labelled / 110 unrepaired of 300 frames
    frac = meta["samples"] / 20000
    assert 0.18 < frac < 0.36, frac
