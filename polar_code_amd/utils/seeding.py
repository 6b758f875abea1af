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
    """Philox key word of one SNR point of a device-generated (--rng philox) sweep.  Points on the
    0.1 dB grid keep round(10 Eb/N0) (the streams of every earlier sweep); any other point gets
    2^31 + round(10^6 Eb/N0) mod 2^31, so grids down to 10^-6 dB never share a stream (two points
    0.05 dB apart used to round to the same word and reuse each other's frames)."""
    t = round(float(snr_db) * 10.0)
    if abs(float(snr_db) * 10.0 - t) < 1e-9:
        return int(t) & 0x7FFFFFFF
    return (1 << 31) | (int(round(float(snr_db) * 1e6)) & 0x7FFFFFFF)


__all__ = ["seed_all", "philox_stream_id"]
