"""Throughput of the exact decodes alone on the headline workload (10^6 frames, (128,64)+CRC-24,
Eb/N0 = 5 dB): every frame on the two-lanes-per-path exact kernel (screening off) or on the exact
lane-per-path instance (PSCL_TUNE_LANE_EXACT = 3), beside the default screening decode.
    python tools/exact_rate.py [L] [steps]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from polar_code_amd import _native  # noqa: E402
from polar_code_amd.polar.polar import construct_info_set  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 8
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
B = 1_000_000
info = construct_info_set(128, 64)
for name in ("screening (default)", "exact kernel only", "exact lane only"):
    dec = _native.Decoder(128, info, L, "0x1864CFB")
    if name == "exact kernel only":
        dec.set_screening(False)
        dec.set_tuning(lane_exact=2)
    elif name == "exact lane only":
        dec.set_tuning(lane_exact=3)
    with _native.DeviceArena(dec) as mem:
        d_llr, d_msg = mem.alloc(B * 128 * 8), mem.alloc(B * 8)
        d_best, d_flags = mem.alloc(B * 8), mem.alloc(B)
        dec.channel_device(0, 50, 5.0, 0.5, 40, 0, B, d_llr, d_msg)
        dec.decode_device(d_llr, B, d_best=d_best, d_flags=d_flags)
        dec.sync()
        t = time.perf_counter()
        for _ in range(steps):
            dec.decode_device(d_llr, B, d_best=d_best, d_flags=d_flags)
        dec.sync()
        ms = (time.perf_counter() - t) * 1e3 / steps
    print(f"L={L} {name}: {ms:.3f} ms per 10^6 frames = {B / ms / 1e3:.1f} M frames/s", flush=True)
    dec.close()
