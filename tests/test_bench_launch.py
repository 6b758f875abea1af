"""bench.py's own rank launcher, on CPU (no GPU here): `--gpus N` without a launcher
environment starts N child ranks and fails as a whole when a rank fails (no hang); a launcher
environment whose WORLD_SIZE disagrees with --gpus is refused before torch is imported."""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(kw)
    return env


def test_world_size_mismatch_refused():
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, capture_output=True, text=True,
                         env=_env(WORLD_SIZE="1"), timeout=60)
    assert res.returncode != 0 and "WORLD_SIZE=1" in res.stderr


def test_launcher_fails_when_ranks_fail():
    # on a host without a GPU every rank fails at device selection; the parent must report it
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                          "--no-cpu-baseline", "--extra", "none"], cwd=ROOT, capture_output=True, text=True,
                         env=_env(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""), timeout=300)
    assert res.returncode != 0
    assert "rank(s) failed" in res.stderr
    assert not [x for x in res.stdout.splitlines() if x.startswith("{")]


def test_launcher_ranks_join_and_exit():
    """The process-group path of the launcher on CPU (PSCL_BENCH_DIST_ONLY: gloo init with the
    explicit timeout, one barrier, no GPU): both ranks join and the job exits 0."""
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, capture_output=True, text=True,
                         env=_env(PSCL_BENCH_DIST_ONLY="1", PSCL_RANK_STALL_S="120"), timeout=300)
    assert res.returncode == 0, res.stderr[-2000:]


def test_launcher_ends_job_when_a_rank_never_joins():
    """Rank 1 never joins the process group (PSCL_BENCH_STALL_RANK): rank 0 waits in
    init_process_group, no rank finishes a stage, and the launcher's watchdog stops both ranks and
    exits non-zero within the stall bound (plus the 30 s SIGTERM grace), never hanging."""
    import time

    t0 = time.time()
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, capture_output=True, text=True,
                         env=_env(PSCL_BENCH_DIST_ONLY="1", PSCL_BENCH_STALL_RANK="1", PSCL_RANK_STALL_S="10",
                                  PSCL_PG_TIMEOUT_S="3600"), timeout=240)
    dt = time.time() - t0
    assert res.returncode != 0
    assert "no rank progressed" in res.stderr, res.stderr[-2000:]
    assert dt < 10 + 30 + 60, dt  # (bound + SIGTERM grace + interpreter start-up)
