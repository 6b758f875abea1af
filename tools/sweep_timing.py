"""Per-SNR wall time of the Philox FER sweep (TX + SCL + DL-SCL + counters on the GPU).

    python tools/sweep_timing.py [M] [frames_per_snr] [batch] [threads] [snr,snr,...]
"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from polar_code_amd.eval import run_fer_sweep as rfs  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 8
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 4_000_000
batch = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 19
streams = int(sys.argv[4]) if len(sys.argv) > 4 else 2
snrs = [float(x) for x in sys.argv[5].split(",")] if len(sys.argv) > 5 else [4.0, 4.5, 5.0, 5.5, 6.0, 6.5]

for rep, snr in enumerate([snrs[0]] + snrs):  # the first pass warms up
    c = np.zeros(rfs.NCOUNT, np.int64)
    args = rfs.build_argparser().parse_args(
        ["--M", str(M), "--frames", str(frames), "--snr_lo", str(snr), "--snr_hi", str(snr), "--snr_step", "0",
         "--retries", "8", "--beta", str(Path(__file__).resolve().parent.parent / "tests" / "golden" / f"beta_M{M}.npy"),
         "--rng", "philox", "--batch", str(batch), "--streams", str(streams), "--include_uncoded",
         "--out_dir", "/tmp/sweep_timing", "--no_plot"])
    t0 = time.perf_counter()
    row = rfs.run_sweep(args)[0]
    dt = time.perf_counter() - t0
    c[rfs.C_SCL_ERR] = round(row["fer_scl"] * frames)
    c[rfs.C_DL_ERR] = round(row["fer_dl"] * frames)
    c[rfs.C_DL_WORK] = round(row["avg_retries"] * frames)
    if rep == 0:
        continue
    print(f"M={M} {snr} dB: {frames / dt / 1e6:.1f} M frames/s, FER scl {c[rfs.C_SCL_ERR] / frames:.3e} "
          f"dl {c[rfs.C_DL_ERR] / frames:.3e}, retries/frame {c[rfs.C_DL_WORK] / frames:.3f}", flush=True)
