"""CRC utilities (host mirror of dl_scl_polar/polar/crc.py:10-59).

The reference divides bit by bit.  CRC is linear over GF(2), so here a message's
remainder is the XOR of precomputed per-position remainders, evaluated as one GF(2)
matrix product for a whole batch.  Same conventions: hex-string polynomial read MSB
first (crc.py:10-16), zero initial value, no reflection, no final XOR.  On the GPU the
same columns drive the decoder's incremental syndrome (csrc/capi.cpp).
"""
from __future__ import annotations

import functools

import numpy as np


def _poly_value(poly) -> int:
    if isinstance(poly, (int, np.integer)):
        return int(poly)
    if not poly:
        raise ValueError("CRC polynomial string must be non-empty")
    return int(poly, 16)


@functools.lru_cache(maxsize=128)
def _remainder_columns(poly_value: int, length: int, divided: int) -> np.ndarray:
    """R[q] = remainder bits of the unit vector e_q (length `length`, first `divided`
    positions divided out as in crc.py:31-35 / :51-55).  Shape [length, degree]."""
    deg = poly_value.bit_length() - 1
    pb = np.array([(poly_value >> (deg - k)) & 1 for k in range(deg + 1)], dtype=np.uint8)
    cols = np.zeros((length, deg), dtype=np.uint8)
    for q in range(length):
        buf = np.zeros(length, dtype=np.uint8)
        buf[q] = 1
        for i in range(divided):
            if buf[i]:
                buf[i : i + deg + 1] ^= pb
        cols[q] = buf[length - deg :]
    return cols


def attach_crc(msg_bits: np.ndarray, poly: str) -> np.ndarray:
    """Append CRC parity bits (crc.py:19-37).  Accepts [k] or a batch [B, k]."""
    msg_bits = np.asarray(msg_bits)
    if msg_bits.ndim not in (1, 2):
        raise ValueError("msg_bits must be a 1D array")
    value = _poly_value(poly)
    deg = value.bit_length() - 1
    if deg <= 0:
        raise ValueError("Polynomial degree must be positive")
    m = msg_bits.astype(np.int8) & 1
    k = m.shape[-1]
    cols = _remainder_columns(value, k + deg, k)[:k]
    rem = (m.astype(np.int64) @ cols.astype(np.int64)) & 1
    return np.concatenate([m, rem.astype(np.int8)], axis=-1)


def crc_syndrome(msg_with_crc: np.ndarray, poly: str) -> np.ndarray:
    """Remainder bits of msg_with_crc ([k] or [B, k]); all-zero <=> CRC passes."""
    m = np.asarray(msg_with_crc).astype(np.int8) & 1
    value = _poly_value(poly)
    deg = value.bit_length() - 1
    k = m.shape[-1]
    if k <= deg:
        raise ValueError("Message too short for the provided CRC polynomial")
    cols = _remainder_columns(value, k, k - deg)
    return (m.astype(np.int64) @ cols.astype(np.int64)) & 1


def check_crc(msg_with_crc: np.ndarray, poly: str):
    """True if msg_with_crc satisfies the CRC (crc.py:40-56).  A batch [B, k] returns [B] bools."""
    msg_with_crc = np.asarray(msg_with_crc)
    if msg_with_crc.ndim not in (1, 2):
        raise ValueError("msg_with_crc must be a 1D array")
    syn = crc_syndrome(msg_with_crc, poly)
    ok = ~syn.any(axis=-1)
    return bool(ok) if msg_with_crc.ndim == 1 else ok


__all__ = ["attach_crc", "check_crc", "crc_syndrome"]
