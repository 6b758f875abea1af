"""Build a variant of the HIP library with extra compile flags (A/B timing, diagnostics).

    python tools/build_variant.py <name> [--spec C_L] [-DFLAG=V ...]   ->  tools/_variant/lib_<name>.so
(--spec C_L: recompile only the scl128_spec instance (code C, list size L) with the flags and
link it with the product build's other objects in polar_code_amd/_build)
Time variants with tools/ab_bench.sh; they are never loaded by the product.
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from polar_code_amd import build as B  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
spec = None
if "--spec" in flags:
    i = flags.index("--spec")
    spec = flags[i + 1]
    flags = flags[:i] + flags[i + 2:]
out = ROOT / "tools" / "_variant"
objdir = out / f"obj_{name}"
objdir.mkdir(parents=True, exist_ok=True)
unit = None
if "--unit" in flags:  # recompile one non-spec source (e.g. scl_long) with the flags
    i = flags.index("--unit")
    unit = flags[i + 1] + ".o"
    flags = flags[:i] + flags[i + 2:]
if spec:
    unit = f"scl128_spec_{spec}.o"
# the variant's own build hash (product hash + its flag set) is compiled into its capi.o, so a
# variant never reports the product's hash (bench.py keys PMC entries by it)
vhash = B.hashlib.sha256((B.source_hash() + "\0" + " ".join([name, spec or "", *flags])).encode()).hexdigest()[:16]
if unit:
    units = B.hip_units(objdir, hash_=vhash)
    mine = [u for u in units if u[2].name == unit or u[0].name == "capi.cpp"]
    objs = B.compile_keyed([u for u in mine if u[0].name != "capi.cpp"], flags)
    objs += B.compile_keyed([u for u in mine if u[0].name == "capi.cpp"], [])
    prod = B.PKG / "_build" / B.ARCH
    rest = [u for u in B.hip_units(prod) if u[2].name != unit and u[0].name != "capi.cpp"]
    objs += B.compile_keyed(rest, [])  # the product's objects, rebuilt if not current
else:
    objs = B.compile_keyed(B.hip_units(objdir, hash_=vhash), flags)
subprocess.check_call([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *objs, "-o", str(out / f"lib_{name}.so")])
print(out / f"lib_{name}.so")
