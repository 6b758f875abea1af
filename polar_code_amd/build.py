"""Build the native parts in-tree.

  polar_code_amd/libpolar_mi355x.so   HIP kernels + C ABI for gfx950 (the product)
  oracle/liboracle_scl.so             C restatement of the reference (test/baseline only)
  oracle/libsoftplus_host.so          host build of csrc/glibc_softplus.h (parity test only)

Run:  python -m polar_code_amd.build   (or __graft_entry__.build()).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
ORACLE = ROOT / "oracle"
LIB = PKG / "libpolar_mi355x.so"
ARCH = os.environ.get("PSCL_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_SOURCES = ["scl_kernels.hip", "scl128.hip", "scl128_spec.hip", "scl128_lane.hip", "scl_lane_long.hip", "scl_long.hip", "dlscl.hip", "capi.cpp",
               "scl_cpu.cpp"]
HIP_DEPS = HIP_SOURCES + ["scl_kernels.h", "scl_device.h", "scl128_impl.h", "glibc_softplus.h", "exp_table.inc"]
# scl128_spec.hip is compiled once per (information-set code, list size): 8 objects
SPEC_UNITS = [(c, l) for c in (1, 2) for l in (1, 2, 4, 8)]


BASE_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wno-unused-result", "-Wno-unused-value"]
HASH_MARK = b"PSCL_BUILD_HASH="


def source_hash(flags: list[str] | None = None) -> str:
    """sha256 (16 hex digits) of every source and header the library is compiled from, the
    target, the compile flags and the unit list.  Embedded in the library (pscl_build_hash)."""
    h = hashlib.sha256()
    h.update(" ".join([ARCH, *BASE_FLAGS, *(flags or []), repr(SPEC_UNITS), *HIP_SOURCES]).encode())
    for f in [*(CSRC / s for s in HIP_DEPS), INCLUDE / "polar_scl.h"]:
        h.update(f.name.encode() + b"\0" + f.read_bytes())
    return h.hexdigest()[:16]


def library_hash(lib: Path = LIB) -> str | None:
    """The hash embedded in a built library (read from its bytes; nothing is loaded)."""
    try:
        data = lib.read_bytes()
    except OSError:
        return None
    i = data.find(HASH_MARK)
    if i < 0:
        return None
    return data[i + len(HASH_MARK): i + len(HASH_MARK) + 16].decode(errors="replace")


def hip_units(objdir: Path, tag: str = "", hash_: str | None = None) -> list[tuple[Path, list[str], Path]]:
    """(source, extra flags, object) for every compile of the HIP library."""
    units = []
    for src in HIP_SOURCES:
        if src == "scl128_spec.hip":
            for c, l in SPEC_UNITS:
                units.append((CSRC / src, [f"-DPSCL_SPEC_CODE={c}", f"-DPSCL_SPEC_LMAX={l}"],
                              objdir / f"scl128_spec_{c}_{l}{tag}.o"))
        else:
            extra = [f'-DPSCL_BUILD_HASH="{hash_}"'] if (src == "capi.cpp" and hash_) else []
            units.append((CSRC / src, extra, objdir / (Path(src).stem + tag + ".o")))
    return units


def compile_units(units, flags: list[str], jobs: int | None = None) -> list[str]:
    """Compile the units in parallel (the spec instances take ~40 s each)."""
    from concurrent.futures import ThreadPoolExecutor

    if not units:
        return []
    base = [HIPCC, f"--offload-arch={ARCH}", *BASE_FLAGS, f"-I{INCLUDE}", f"-I{CSRC}", *flags]
    jobs = jobs or min(len(units), max(1, min(16, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(lambda u: _run([*base, *u[1], "-c", str(u[0]), "-o", str(u[2])]), units))
    return [str(u[2]) for u in units]


def _run(cmd: list[str]) -> None:
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError(f"build step failed: {' '.join(cmd)}")


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def unit_key(unit, flags: list[str]) -> str:
    """Content key of one object: target, compiler, every flag (base, unit, extra) and the bytes
    of its source and of every header it may include.  Stored next to the object
    (<obj>.key) so an object is reused only when it was built from exactly these inputs
    (modification times and the shared object directory are not trusted)."""
    h = hashlib.sha256()
    h.update("\0".join([ARCH, HIPCC, *BASE_FLAGS, *unit[1], *flags]).encode())
    headers = sorted([*CSRC.glob("*.h"), *CSRC.glob("*.inc"), *INCLUDE.glob("*.h")])
    for f in [unit[0], *headers]:
        h.update(f.name.encode() + b"\0" + f.read_bytes())
    return h.hexdigest()[:32]


def _key_path(obj: Path) -> Path:
    return obj.with_name(obj.name + ".key")


def object_current(unit, flags: list[str]) -> bool:
    kp = _key_path(unit[2])
    return unit[2].exists() and kp.exists() and kp.read_text().strip() == unit_key(unit, flags)


def compile_keyed(units, flags: list[str], force: bool = False) -> list[str]:
    """Compile every unit whose key differs from the one recorded with its object."""
    todo = [u for u in units if force or not object_current(u, flags)]
    for u in todo:
        _key_path(u[2]).unlink(missing_ok=True)
    compile_units(todo, flags)
    for u in todo:
        _key_path(u[2]).write_text(unit_key(u, flags) + "\n")
    return [str(u[2]) for u in units]


def build_hip(force: bool = False) -> Path:
    """Rebuild unless the library's embedded hash equals the hash of the sources in the tree
    (modification times are not trusted: a copied or pushed library may look newer).  Objects
    are reused only when their recorded content key (ARCH, flags, source and headers) matches."""
    want = source_hash()
    if not force and library_hash() == want:
        return LIB
    objdir = PKG / "_build" / ARCH
    objdir.mkdir(parents=True, exist_ok=True)
    units = hip_units(objdir, hash_=want)
    objs = compile_keyed(units, [], force)
    tmp = LIB.with_suffix(".so.tmp")
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", str(tmp)])
    os.replace(tmp, LIB)
    return LIB


def build_oracle(force: bool = False) -> list[Path]:
    out = []
    lib = ORACLE / "liboracle_scl.so"
    src = ORACLE / "scl_oracle.c"
    if force or _stale(lib, [src]):
        _run(["gcc", "-O2", "-fPIC", "-shared", "-fopenmp", "-ffp-contract=off", "-fno-builtin",
              str(src), "-o", str(lib), "-lm"])
    out.append(lib)
    sp = ORACLE / "libsoftplus_host.so"
    spsrc = ORACLE / "softplus_host.c"
    if force or _stale(sp, [spsrc, CSRC / "glibc_softplus.h", CSRC / "exp_table.inc"]):
        _run(["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", f"-I{CSRC}", str(spsrc), "-o", str(sp), "-lm"])
    out.append(sp)
    return out


def build_all(force: bool = False) -> None:
    build_hip(force)
    build_oracle(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print(LIB)
