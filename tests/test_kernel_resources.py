"""The kernels on the default decode paths use no scratch (CPU test: reads the gfx950 code objects'
metadata in the built library, tools/kernel_resources.py).  A kernel with scratch costs private
memory traffic and makes the runtime allocate a queue's scratch at its first dispatch there, which
stalled the first retry decode of a DL-SCL chain by ~130 us."""
import importlib.util
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
LIB = ROOT / "polar_code_amd" / "libpolar_mi355x.so"
READELF = Path("/opt/rocm/lib/llvm/bin/llvm-readelf")

# mangled-name patterns of the hot kernels: the lane-per-path screening kernels (plain and forced
# bits at N = 128; the runtime-information-set kernel at N = 128..1024, L = 4..32), the exact
# N = 128 re-decode / forced-bit instances (HIST = CH = APX = false, compiled-in code 1 or 2), the
# DL-SCL post pass, the exact long-code kernel (the re-decode of deferred N >= 256 frames).  The
# opt-in fused instances of the lane kernel (TXF: fused TX, FP: fused post pass; off by default,
# DESIGN.md §5.4-5.5) are not on a default path: they spill (profiles/r06e, r06l)
HOT = [r"scl_lane_kernelILi[48]ELi[12]ELb[01]ELb0ELb0E",
       r"scl_lane_long_kernelILi(7|8|9|10)ELi(4|8|16|32)E",
       r"scl128_kernelILi[48]ELb0ELb0ELb[01]ELi1ELb0E",
       r"dl_post_kernelILi128ELi(64|88)ELi4E",
       r"scl_long_kernelILi(4|8|16|32)ELb[01]E"]


def _kernels():
    spec = importlib.util.spec_from_file_location("kernel_resources", ROOT / "tools" / "kernel_resources.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.kernels(LIB)


@pytest.mark.skipif(not LIB.exists() or not READELF.exists(), reason="needs the built library and llvm-readelf")
def test_hot_kernels_use_no_scratch():
    ks = _kernels()
    for pat in HOT:
        hits = {n: v for n, v in ks.items() if re.search(pat, n)}
        assert hits, f"no kernel matches {pat}"
        for n, v in hits.items():
            assert v.get("private_segment_fixed_size", 0) == 0, f"{n} uses {v['private_segment_fixed_size']} B of scratch"
            assert v.get("vgpr_spill_count", 0) == 0, f"{n} spills {v['vgpr_spill_count']} VGPRs"
