"""Polar code primitives (mirror of dl_scl_polar/polar/polar.py).

  construct_info_set   host constant (Gaussian approximation, polar.py:37-103)
  encode / _polar_transform   host bit transforms (polar.py:17-29,106-119), batch-capable;
                       the GPU TX chain has its own in-register transform (csrc/scl_kernels.hip)
  sc_decode            successive cancellation ON THE GPU (pscl_sc_decode; polar.py:130-168)
"""
from __future__ import annotations

import functools
import math

import numpy as np

from .. import config
from .. import _native


def _check_power_of_two(n: int) -> None:
    if n <= 0 or (n & (n - 1)) != 0:
        raise ValueError("N must be a power of two")


def _polar_transform(u: np.ndarray) -> np.ndarray:
    """Arikan transform x = u G_N, natural order (polar.py:17-29).  u: [..., N] bits."""
    x = np.array(u, copy=True)
    N = x.shape[-1]
    _check_power_of_two(N)
    lead = x.shape[:-1]
    step = 1
    while step < N:
        v = x.reshape(*lead, N // (2 * step), 2, step)
        v[..., 0, :] ^= v[..., 1, :]
        step *= 2
    return x


def _polarization_weights(N: int) -> np.ndarray:
    n = int(math.log2(N))
    idx = np.arange(N)
    w = np.zeros(N, dtype=float)
    for j in range(n):
        w += ((idx >> j) & 1) * 2 ** (j / 4.0)
    return w


def _phi_inv(x: float) -> float:
    if x > 12.0:
        return 0.9861 * x - 2.3152
    if x > 3.5:
        return x * (0.009005 * x + 0.7694) - 0.9507
    if x > 1.0:
        return x * (0.062883 * x + 0.3678) - 0.1627
    return x * (0.2202 * x + 0.06448)


def _gaussian_pe(N: int, K: int, design_snr_db: float) -> np.ndarray:
    """Mean-LLR recursion and Q-function error probabilities (polar.py:61-82)."""
    rate = K / N
    sigma_sq = 1.0 / (2.0 * rate * 10 ** (design_snr_db / 10.0))
    m = [0.0] * N
    m[0] = 2.0 / sigma_sq
    for level in range(1, int(math.log2(N)) + 1):
        half = (1 << level) >> 1
        for j in range(half):
            t = m[j]
            m[j] = _phi_inv(t)
            m[half + j] = 2.0 * t
    return np.array([0.5 - 0.5 * math.erf(math.sqrt(max(v, 1e-12)) / 2.0) for v in m])


@functools.lru_cache(maxsize=None)
def _info_set_cached(N: int, K: int, method: str, design_snr_db: float) -> tuple:
    _check_power_of_two(N)
    if not (0 < K <= N):
        raise ValueError("K must satisfy 0 < K <= N")
    if method == "polarization":
        order = np.argsort(_polarization_weights(N), kind="stable")
    elif method == "gaussian":
        order = np.argsort(_gaussian_pe(N, K, design_snr_db), kind="stable")
    else:
        raise ValueError(f"Unsupported construction method: {method}")
    return tuple(np.sort(order[:K]).tolist())


def construct_info_set(N: int, K: int, method: str = "gaussian", design_snr_db: float = 2.5) -> np.ndarray:
    """Sorted information-set indices of an (N, K) polar code (polar.py:85-103)."""
    return np.array(_info_set_cached(int(N), int(K), method, float(design_snr_db)), dtype=np.int32)


def encode(msg_bits: np.ndarray) -> np.ndarray:
    """Encode K message bits with the default (N, K) code (polar.py:106-119).
    Accepts [K] or a batch [B, K]."""
    cfg = config.DEFAULTS
    msg_bits = np.asarray(msg_bits)
    if msg_bits.ndim not in (1, 2):
        raise ValueError("msg_bits must be 1D")
    if msg_bits.shape[-1] != cfg.K:
        raise ValueError(f"msg_bits must have length {cfg.K}")
    info_set = construct_info_set(cfg.N, cfg.K)
    u = np.zeros(msg_bits.shape[:-1] + (cfg.N,), dtype=np.int8)
    u[..., info_set] = msg_bits.astype(np.int8) & 1
    return _polar_transform(u)


def sc_decode(llr: np.ndarray, info_set: np.ndarray, *, device: int = 0) -> np.ndarray:
    """SC decoding with hard decisions (polar.py:130-168), run on the GPU.
    llr: [N] (returns [K] int8) or a batch [B, N] (returns [B, K])."""
    llr = np.asarray(llr)
    if llr.ndim not in (1, 2):
        raise ValueError("llr must be 1D")
    N = llr.shape[-1]
    _check_power_of_two(N)
    info_set = np.asarray(info_set)
    if info_set.ndim != 1:
        raise ValueError("info_set must be 1D")
    if np.any(info_set < 0) or np.any(info_set >= N):
        raise ValueError("info_set indices out of range")
    dec = _native.get_decoder(N, info_set, 1, None, device)
    bits = dec.sc_decode(llr.astype(np.float64))
    return bits[0] if llr.ndim == 1 else bits


def _f(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Min-sum check node (polar.py:122-123); host helper kept for API parity."""
    return np.sign(a) * np.sign(b) * np.minimum(np.abs(a), np.abs(b))


def _g(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    """Variable node (polar.py:126-127); host helper kept for API parity."""
    return b + (1 - 2 * c) * a


__all__ = ["construct_info_set", "encode", "sc_decode"]
