"""NR polar rate matching (mirror of dl_scl_polar/nr/polar/rate_match.py).

Host-side utilities; the decode path runs de-rate-matching inside the GPU decode kernel."""
from __future__ import annotations

import numpy as np


def rate_match_polar(bits: np.ndarray, E: int, mode: str = "puncture") -> np.ndarray:
    """rate_match.py:8-16: truncate (E <= N) or repeat cyclically to E."""
    bits = np.asarray(bits)
    if bits.ndim != 1:
        raise ValueError("bits must be 1D")
    N = bits.size
    if E <= N:
        return bits[:E]
    return np.resize(bits, E)


def derate_match_polar(bits_E: np.ndarray, N: int, mode: str = "puncture") -> np.ndarray:
    """rate_match.py:19-39: E <= N pads with -1.0; E > N averages the repeats (summed in
    transmission order, then divided by the repeat count)."""
    bits_E = np.asarray(bits_E)
    if bits_E.ndim != 1:
        raise ValueError("bits_E must be 1D")
    if bits_E.size <= N:
        result = np.full(N, fill_value=-1.0, dtype=np.float64)
        result[: bits_E.size] = bits_E
        return result
    reps, remainder = divmod(bits_E.size, N)
    accum = np.zeros(N, dtype=np.float64)
    counts = np.full(N, reps, dtype=np.int32)
    accum += bits_E[: reps * N].reshape(reps, N).sum(axis=0)
    if remainder:
        accum[:remainder] += bits_E[reps * N :]
        counts[:remainder] += 1
    return accum / counts


__all__ = ["rate_match_polar", "derate_match_polar"]
