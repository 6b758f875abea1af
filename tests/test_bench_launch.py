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
