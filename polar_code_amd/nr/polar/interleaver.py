"""Simplified NR sub-block interleaver (mirror of dl_scl_polar/nr/polar/interleaver.py).

Host-side array utilities; the decode path applies the inverse permutation inside the GPU
decode kernel (pscl_set_rate_match)."""
from __future__ import annotations

import functools

import numpy as np

_INTERLEAVER_BLOCK = 32


@functools.lru_cache(maxsize=64)
def _order(total: int) -> np.ndarray:
    nb = total // _INTERLEAVER_BLOCK
    i = np.arange(total)
    return ((i % _INTERLEAVER_BLOCK) * nb + i // _INTERLEAVER_BLOCK).astype(np.int32)


def subblock_interleave(bits: np.ndarray, mode: str = "default") -> np.ndarray:
    """interleaver.py:10-23: pad to a multiple of 32 with -1, read column-wise."""
    bits = np.asarray(bits)
    if bits.ndim != 1:
        raise ValueError("bits must be 1D")
    total = -(-bits.size // _INTERLEAVER_BLOCK) * _INTERLEAVER_BLOCK
    padded = np.full(total, fill_value=-1, dtype=bits.dtype)
    padded[: bits.size] = bits
    return padded[_order(total)]


def subblock_deinterleave(bits: np.ndarray, original_len: int, mode: str = "default") -> np.ndarray:
    """interleaver.py:26-37: inverse permutation, truncated to original_len."""
    bits = np.asarray(bits)
    if bits.ndim != 1:
        raise ValueError("bits must be 1D")
    total = -(-original_len // _INTERLEAVER_BLOCK) * _INTERLEAVER_BLOCK
    padded = np.zeros(total, dtype=bits.dtype)
    padded[: bits.size] = bits
    out = np.empty(total, dtype=bits.dtype)
    out[_order(total)] = padded
    return out[:original_len]


__all__ = ["subblock_interleave", "subblock_deinterleave"]
