"""The bench's config-3 sweep alone (bench.py config3_sweep): run_fer_sweep --rng philox, L = 8,
4.0-6.5 dB, 10^6 frames per point, after an untimed 4.0-5.5 dB warm-up at another seed (four
pipelined calls: every scratch set and chain set of the handle used once, as in the bench, whose
5 dB point follows its 6-point sweep); prints the wall time of the timed pass (for rocprofv3
traces of the product path).

    python tools/config3_run.py [frames] [lo] [hi] [k=v,k=v] [batch]   (handle tuning knobs and the
    frames per pscl_simulate_device call, run_fer_sweep --batch: A/B only; "-" for no knobs)
"""
import contextlib
import io
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

from polar_code_amd.eval import run_fer_sweep as rfs  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
lo = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
hi = float(sys.argv[3]) if len(sys.argv) > 3 else 6.5
tune = (dict((k, int(v)) for k, v in (kv.split("=") for kv in sys.argv[4].split(",")))
        if len(sys.argv) > 4 and sys.argv[4] not in ("", "-") else {})
batch = int(sys.argv[5]) if len(sys.argv) > 5 else 0
if tune:  # the sweep's cached handle (run_fer_sweep: get_decoder(N, info, M, crc, device))
    from polar_code_amd import _native
    from polar_code_amd.polar.polar import construct_info_set
    _native.get_decoder(128, construct_info_set(128, 64), 8, "0x1864CFB", 0).set_tuning(**tune)


def run(a_lo, a_hi, seed, td):
    a = rfs.build_argparser().parse_args(
        ["--M", "8", "--frames", str(frames), "--snr_lo", f"{a_lo:g}", "--snr_hi", f"{a_hi:g}", "--snr_step", "0.5",
         "--retries", "8", "--beta", str(ROOT / "tests" / "golden" / "beta_M8.npy"), "--rng", "philox",
         "--include_uncoded", "--no_plot", "--seed", str(seed), "--out_dir", td, "--plot_dir", td]
        + (["--batch", str(batch)] if batch else []))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        rows = rfs.run_sweep(a)
    torch.cuda.synchronize()
    return rows, time.perf_counter() - t0


with tempfile.TemporaryDirectory() as td:
    run(4.0, 5.5, 1, td)
    rows, t = run(lo, hi, 0, td)
print(f"config 3 sweep {lo:g}-{hi:g} dB{' ' + str(tune) if tune else ''}{f' batch {batch}' if batch else ''}: {len(rows)} points x {frames} frames in {t * 1e3:.2f} ms = "
      f"{len(rows) * frames / t / 1e6:.1f} M frames/s", flush=True)
