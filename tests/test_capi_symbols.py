"""The C-ABI library loads and exports every symbol include/polar_scl.h declares (no GPU)."""
import re
from pathlib import Path

import pytest

from polar_code_amd import _native

HEADER = Path(__file__).resolve().parent.parent / "include" / "polar_scl.h"


def _declared():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pscl_[a-z0-9_]+)\s*\(", text)))


def test_header_matches_binding_table():
    assert _declared() == sorted(_native.EXPORTS)


def test_library_exports_all_symbols():
    lib = _native.lib()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.pscl_abi_version() == 1


def test_no_gpu_fails_loudly():
    if _native.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(_native.PolarNativeError):
        _native.Decoder(128, list(range(64, 128)), 8, "0x1864CFB")


def test_argument_errors_map_to_reference_exceptions():
    # argument validation happens before any device call
    with pytest.raises(ValueError):
        _native.Decoder(100, [1, 2], 4, None)
    with pytest.raises(ValueError):
        _native.Decoder(128, [1, 2], 0, None)
    with pytest.raises(ValueError):
        _native.Decoder(128, list(range(10)), 4, "0x1864CFB")  # K <= CRC degree
    with pytest.raises(NotImplementedError):
        _native.Decoder(2048, list(range(10)), 4, None)  # N > PSCL_MAX_N = 1024
