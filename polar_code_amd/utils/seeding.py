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


__all__ = ["seed_all"]
