"""Timing-only ablation of the decode kernel (diagnostic builds, outputs are NOT valid).

  python tools/ablate.py build          # builds tools/_ablate/lib_<mask>.so
  python tools/ablate.py run <mask>     # times one build (separate process per build)
mask bits: 1 = no softplus, 2 = no rank/sort, 4 = no LLR tree updates, 8 = no fused depth-1..3
recompute, 16 = no frozen-phase re-rank, 32 = no survivor gathers, 64 = no epilogue bit gather,
128 = no leaf f/g.
  rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES -- python tools/ablate.py run <mask>   # dynamic counts
"""
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "tools" / "_ablate"
MASKS = [int(m) for m in os.environ.get("MASKS", "0 1 2 4 8 16 7").split()]


def build():
    sys.path.insert(0, str(ROOT))
    from polar_code_amd import build as B

    OUT.mkdir(exist_ok=True)
    for m in MASKS:
        objs = B.compile_units(B.hip_units(OUT, f"_{m}"), [f"-DPSCL_ABLATE={m}"])
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o",
                               str(OUT / f"lib_{m}.so")])


def run(mask, L=8, B=1_000_000):
    os.environ["PSCL_LIB_PATH"] = str(OUT / f"lib_{mask}.so")
    sys.path.insert(0, str(ROOT))
    import torch
    from polar_code_amd import _native
    from polar_code_amd.polar.polar import construct_info_set

    dec = _native.Decoder(128, construct_info_set(128, 64), L, "0x1864CFB")
    dec.set_stream(torch.cuda.current_stream().cuda_stream)
    llr = torch.empty((B, 128), dtype=torch.float64, device="cuda")
    msg = torch.empty((B, 1), dtype=torch.int64, device="cuda")
    best = torch.empty((B, 1), dtype=torch.int64, device="cuda")
    dec.channel_device(0, 50, 5.0, 0.5, 40, 0, B, llr.data_ptr(), msg.data_ptr())
    dec.decode_device(llr.data_ptr(), B, d_best=best.data_ptr())
    torch.cuda.synchronize()
    dec.timing_enable(True)
    for _ in range(3):
        dec.decode_device(llr.data_ptr(), B, d_best=best.data_ptr())
    n, ms = dec.timing_read()
    print(f"ablate mask={mask} L={L}: {ms / n:.2f} ms per {B} frames", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 8)
