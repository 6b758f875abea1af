"""run_ber_sweep mirror: stream replay across SNR points, the data-dependent stop rule and the
CSV rows, against the reference's own rows (tests/golden/g11_ber.npz).

CPU: the GPU decoder is swapped for the oracle (test infrastructure); everything else --
stream, batching, exact stop, rewinds, NR host front-end, CSV -- is the product code.
"""
import numpy as np
import pytest

import oracle
from polar_code_amd.eval import run_ber_sweep as rb
from polar_code_amd.nr.polar import derate_match_polar, subblock_deinterleave

from conftest import GOLDEN

CONFIGS = ["ber_polar_small", "ber_polar_128", "ber_dl_128", "ber_nr_256", "ber_nr_small"]


def _argv(g, name, out):
    argv = str(g[name + "_argv"]).split()
    return [str(GOLDEN / "beta_M4.npy") if a == "BETA4" else a for a in argv] + ["--out", str(out), "--batch", "37"]


def _oracle_decode(self, llr):
    a = self.args
    crc = a.crc_poly if a.K_crc else None
    if a.scheme == "nr_polar_scl":
        llr = np.stack([subblock_deinterleave(derate_match_polar(x, self.N), self.N) for x in llr])
        crc = a.crc_poly
    bits, ok = oracle.decode_batch(llr, self.info_set, a.M, crc)
    work = np.zeros(llr.shape[0])
    if a.scheme == "dl_scl":
        for f in np.flatnonzero(~ok):
            r = oracle.decode_with_retries(llr[f], self.info_set, a.M, a.retries, crc=crc, beta=self.beta)
            bits[f] = r["bits"]
            work[f] = r["attempts"] - 1
    return bits, work


@pytest.mark.parametrize("name", CONFIGS)
def test_rows_match_reference_with_oracle(golden, name, tmp_path, monkeypatch):
    g = golden("g11_ber.npz")
    monkeypatch.setattr(rb._Scheme, "decode", _oracle_decode)
    out = tmp_path / "x.csv"
    rb.main(_argv(g, name, out))
    assert out.read_text() == str(g[name])


def test_payload_bit_errors_ignores_crc_only():
    # reference tests/test_ber_eval.py:7-20, restated
    payload = np.array([0, 1, 1, 0], dtype=np.int8)
    candidate = np.concatenate([payload, np.array([1, 0, 0, 1], dtype=np.int8)])
    candidate[-1] ^= 1
    assert rb._payload_bit_errors(payload, candidate, payload.size) == 0
    assert rb._payload_bit_errors(np.array([0, 1, 0], np.int8), None, 3) == 3


def test_arg_rules():
    with pytest.raises(ValueError):
        rb.parse_args(["--scheme", "dl_scl", "--K_payload", "8", "--K_crc", "4", "--E", "16", "--EbN0_lo", "5",
                       "--EbN0_hi", "5", "--out", "x.csv"])
    args = rb.parse_args(["--scheme", "nr_ldpc", "--K_payload", "6", "--K_crc", "0", "--E", "12", "--EbN0_lo", "5",
                          "--EbN0_hi", "5", "--out", "x.csv"])
    with pytest.raises(NotImplementedError):
        rb.run(args)
