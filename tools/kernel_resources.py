"""Register, spill and scratch figures of every kernel in the built library, read from the gfx950
code objects' metadata notes (no GPU needed).

    python tools/kernel_resources.py [library] [--scratch]     (--scratch: only kernels with scratch)

The code objects sit in clang offload bundles inside the shared library (magic
__CLANG_OFFLOAD_BUNDLE__: entry count, then per entry offset, size and target triple); each
amdgcn entry is an ELF whose NT_AMDGPU_METADATA note llvm-readelf prints as YAML-like text.
"""
import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
LLVM = Path("/opt/rocm/lib/llvm/bin")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
FIELDS = ("private_segment_fixed_size", "vgpr_count", "vgpr_spill_count", "sgpr_spill_count",
          "group_segment_fixed_size")


def code_objects(lib: Path):
    d = lib.read_bytes()
    i = d.find(MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", d, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", d, p)
            p += 24
            triple = d[p:p + tl].decode(errors="replace")
            p += tl
            if "amdgcn" in triple:
                yield d[i + off:i + off + size]
        i = d.find(MAGIC, i + 1)


def kernels(lib: Path):
    """{mangled name: {field: int}} over every code object of the library."""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(code_objects(lib)):
            f = Path(td) / f"co{k}.elf"
            f.write_bytes(co)
            notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(f)], capture_output=True,
                                   text=True, check=True).stdout
            cur = None
            for line in notes.splitlines():
                m = re.match(r"\s+\.name:\s+(\S+)", line)
                if m and not m.group(1).endswith(".kd"):
                    cur = out.setdefault(m.group(1), {})
                    continue
                m = re.match(r"\s+\.(\w+):\s+(\d+)\s*$", line)
                if m and cur is not None and m.group(1) in FIELDS:
                    cur[m.group(1)] = int(m.group(2))
    return out


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    except OSError:
        return list(names)
    return r.stdout.splitlines() if r.returncode == 0 else list(names)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = Path(args[0]) if args else ROOT / "polar_code_amd" / "libpolar_mi355x.so"
    ks = kernels(lib)
    names = sorted(ks)
    for n, dn in zip(names, demangle(names)):
        v = ks[n]
        if "--scratch" in sys.argv and not v.get("private_segment_fixed_size"):
            continue
        dn = dn.replace("(anonymous namespace)::", "").split("(")[0]
        print(f"scratch {v.get('private_segment_fixed_size', 0):4d} B  vgpr {v.get('vgpr_count', 0):3d}  "
              f"vspill {v.get('vgpr_spill_count', 0):3d}  sspill {v.get('sgpr_spill_count', 0):3d}  {dn}")


if __name__ == "__main__":
    main()
