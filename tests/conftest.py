"""Shared pytest setup: marker registration, repo on sys.path, native builds."""
from __future__ import annotations

import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "golden"
for p in (ROOT, ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    # the oracle (test infrastructure) is built from oracle/*.c with gcc; cheap and idempotent
    from polar_code_amd import build as _b

    _b.build_oracle()


def load_golden(name: str):
    import numpy as np

    return np.load(GOLDEN / name, allow_pickle=False)


@pytest.fixture(scope="session")
def golden():
    return load_golden
