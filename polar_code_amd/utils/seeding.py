"""Deterministic seeding (mirror of dl_scl_polar/utils/seeding.py:21-31).

Unlike the reference, importing this module does not pin OMP/torch to one thread: the
decoder runs on the GPU and the host side is not a bottleneck.
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np


def seed_all(seed: int, deterministic_torch: bool = False) -> None:
    """Seed Python, NumPy's legacy global RNG and (if imported) PyTorch."""
    os.environ["PYTHONHASHSEED"] = str(seed)
    random.seed(seed)
    np.random.seed(seed)
    torch = sys.modules.get("torch")
    if torch is not None:
        torch.manual_seed(seed)
        if deterministic_torch:
            torch.use_deterministic_algorithms(True)


def philox_stream_id(snr_db: float) -> int:
    """Philox key word (32 bits) of one SNR point of a device-generated (--rng philox) sweep.

    * Points on the 0.1 dB grid keep their historical word round(10 Eb/N0) mod 2^32 (the streams
      of every earlier sweep, negative points included: -1.0 dB -> 0xFFFFFFF6).  For |Eb/N0| below
      10^8 dB these words lie in [0, 2^30) (non-negative points) or [3 * 2^30, 2^32) (negative ones).
    * Any other point gets 2^31 + (round(10^6 Eb/N0) mod 2^30), inside [2^31, 3 * 2^30), a range no
      grid word reaches, so an off-grid point never shares a stream with a grid point, and two
      off-grid points share one only when they differ by a multiple of 2^30 / 10^6 (~1074 dB).
      (Non-negative off-grid points below that keep the words they had before this layout.)"""
    x = float(snr_db) * 10.0
    t = round(x)
    if abs(x - t) < 1e-9:
        return int(t) & 0xFFFFFFFF
    return (1 << 31) | (int(round(float(snr_db) * 1e6)) & 0x3FFFFFFF)


__all__ = ["seed_all", "philox_stream_id"]
