"""Diagnostic: the rate-matched L = 8 history decode (info_llrs, candidates, metrics) and the
path-LLR replay, each against the oracle on de-rate-matched rows (tests/test_gpu_parity.py's
replay case, split by side).  Run under PSCL_LIB_PATH variants."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "oracle"))
import oracle  # noqa: E402
from polar_code_amd import _native  # noqa: E402
from polar_code_amd.nr.polar import derate_match_polar, subblock_deinterleave  # noqa: E402
from polar_code_amd.polar.polar import construct_info_set  # noqa: E402

N, K, L, E, B = 128, 64, 8, 200, 64
rng = np.random.default_rng(N * 1000 + K + L + E)
info = construct_info_set(N, K)
llr = rng.normal(1.0, 2.5, size=(B, E)) * rng.choice([1.0, -1.0], size=(B, E))
dec = _native.Decoder(N, info, L, "0x1864CFB")
dec.set_rate_match(E)
out = dec.decode(llr, want_metrics=True)
internal = np.stack([subblock_deinterleave(derate_match_polar(x, N), N) for x in llr])
bad_c = bad_m = bad_il = 0
for f in range(B):
    n, c, m, il, b = oracle.decode_scl(internal[f], info, L, crc="0x1864CFB")
    bad_c += int(not np.array_equal(out["cands"][f, :n], c[:n]))
    bad_m += int(not np.array_equal(out["metrics"][f, :n], m[:n]))
    bad_il += int(not np.array_equal(out["info_llrs"][f, :n], il[:n]))
print(f"decoder vs oracle: frames with wrong candidates {bad_c}, metrics {bad_m}, info_llrs {bad_il} (of {B})")
rows = np.repeat(np.arange(B), L)
valid = (np.arange(L)[None, :] < out["n_paths"][:, None]).ravel()
cands = out["cands"].reshape(B * L, K)[valid]
got = dec.path_llrs(llr[rows[valid]], cands)
ref = []
for f in range(B):
    n, c, m, il, b = oracle.decode_scl(internal[f], info, L, crc="0x1864CFB")
    ref.append(il[:n])
ref = np.concatenate(ref)
print(f"replay vs oracle info_llrs: {int((got.view(np.uint64) != ref.view(np.uint64)).any(axis=1).sum())} of {len(ref)} paths differ")
