"""Diagnostics of the long-code kernel against the oracle on one frame (GPU box)."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "oracle"))
import oracle  # noqa: E402
from polar_code_amd import _native  # noqa: E402
from polar_code_amd.polar.polar import construct_info_set  # noqa: E402

np.set_printoptions(linewidth=160, precision=6)
for N, K, M in [(256, 128, 1), (256, 128, 4)]:
    info = construct_info_set(N, K)
    rng = np.random.default_rng(1)
    llr = rng.normal(2.0, 2.0, size=(2, N))
    dec = _native.Decoder(N, info, M, None)
    out = dec.decode(llr)
    n, c, m, il, b = oracle.decode_scl(llr[0], info, M)
    print(f"N={N} M={M}: n_paths gpu {out['n_paths'][0]} oracle {n}")
    print(" metrics gpu", out["metrics"][0][:n], "oracle", m[:n])
    print(" cands gpu   ", out["cands"][0, 0, :40])
    print(" cands oracle", c[0, :40])
    print(" illr gpu   ", out["info_llrs"][0, 0, :8])
    print(" illr oracle", il[0, :8])
    sc = dec.sc_decode(llr)[0] if M == 1 else None
    if sc is not None:
        print(" sc gpu   ", sc[:40])
        print(" sc oracle", oracle.sc_decode(llr[0], info)[:40])
