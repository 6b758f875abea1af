"""Build a variant of the HIP library with extra compile flags (A/B timing, diagnostics).

    python tools/build_variant.py <name> [-DFLAG=V ...]   ->  tools/_variant/lib_<name>.so
Time variants with tools/ab_bench.sh; they are never loaded by the product.
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from polar_code_amd import build as B  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
out = ROOT / "tools" / "_variant"
objdir = out / f"obj_{name}"
objdir.mkdir(parents=True, exist_ok=True)
objs = B.compile_units(B.hip_units(objdir), flags)
subprocess.check_call([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *objs, "-o", str(out / f"lib_{name}.so")])
print(out / f"lib_{name}.so")
