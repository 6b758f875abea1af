"""GPU rehearsal of the multi-rank product path on one MI355X.

Two fresh child processes (subprocess, never an exec of the test process) share the GPU
(PSCL_SHARE_GPU=1) and talk over gloo: the same sharding and counter all-reduces as the
RCCL runs on an 8-GPU node, with the Philox channel and the device DL-SCL retry loop.
  (a) run_fer_sweep --rng philox --dl_engine device at world 2 writes the same CSV as world 1;
  (b) bench.py at world 2 counts 2*B*steps frames and the same frame errors as world 1 over
      the same global frame range.
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(world, argv, timeout=240):
    """world ranks of `python argv...` with torchrun's environment; returns their stdouts."""
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PSCL_SHARE_GPU="1", PSCL_DIST_BACKEND="gloo",
                   PYTHONPATH=str(ROOT) + os.pathsep + os.environ.get("PYTHONPATH", ""))
        procs.append(subprocess.Popen([sys.executable, *argv], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out)
            assert p.returncode == 0, out[-3000:]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return outs


def test_fer_sweep_philox_world2_equals_world1(tmp_path):
    args = ["-m", "polar_code_amd.eval.run_fer_sweep", "--M", "4", "--frames", "120001", "--snr_lo", "3.5",
            "--snr_hi", "4.5", "--snr_step", "0.5", "--retries", "8", "--beta", str(GOLDEN / "beta_M4.npy"),
            "--rng", "philox", "--dl_engine", "device", "--batch", "40000", "--include_uncoded", "--no_plot"]
    csv = {}
    for world in (1, 2):
        d = tmp_path / f"w{world}"
        _launch(world, args + ["--out_dir", str(d), "--plot_dir", str(d)])
        csv[world] = (d / "fer_M4.csv").read_text()
    assert csv[1] == csv[2] and csv[1].count("\n") == 4


def test_bench_world2_counts_every_frame_once():
    B = 50_000
    base = ["bench.py", "--frames", str(B), "--warmup", "1", "--no-cpu-baseline", "--extra", "none"]
    line = {}
    for world, steps in ((1, 4), (2, 2)):  # the same global frames [0, 4B): rank r owns [2rB, 2rB + 2B)
        out = _launch(world, base + ["--steps", str(steps), "--gpus", str(world)])
        line[world] = json.loads([x for x in out[0].splitlines() if x.startswith("{")][-1])
    assert line[2]["n_gpus"] == 2 and line[2]["fer"]["frames"] == 2 * B * 2
    assert line[1]["fer"]["frames"] == 4 * B
    for k in ("frame_errors", "ber", "payload_fer", "payload_ber"):
        assert line[1]["fer"][k] == line[2]["fer"][k], k


def test_bench_gpus2_launches_its_own_ranks():
    """`python bench.py --gpus 2` with no launcher environment (what the driver runs) starts two
    rank processes itself (rank 0 relays its line) and decodes the same global frames as the
    world-1 run over [0, 4B)."""
    B = 50_000
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(PSCL_SHARE_GPU="1", PSCL_DIST_BACKEND="gloo")
    base = [sys.executable, "bench.py", "--frames", str(B), "--warmup", "1", "--no-cpu-baseline", "--extra", "none"]
    line = {}
    for gpus, steps in ((1, 4), (2, 2)):
        res = subprocess.run(base + ["--steps", str(steps), "--gpus", str(gpus)], cwd=ROOT, env=env,
                             capture_output=True, text=True, timeout=240)
        assert res.returncode == 0, (res.stdout + res.stderr)[-3000:]
        lines = [x for x in res.stdout.splitlines() if x.startswith("{")]
        assert len(lines) == 1, res.stdout[-2000:]  # one JSON line: rank 0's
        line[gpus] = json.loads(lines[0])
    assert line[2]["n_gpus"] == 2 and line[2]["fer"]["frames"] == 2 * B * 2
    assert line[1]["fer"]["frames"] == 4 * B
    for k in ("frame_errors", "ber", "payload_fer", "payload_ber"):
        assert line[1]["fer"][k] == line[2]["fer"][k], k


def _world1(argv, group: bool, timeout=240):
    """One process of `python argv...`: with a world-1 launcher environment (a process group on
    the default backend, nccl = RCCL on this GPU) or with none (no group).  Returns its output."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                            "MASTER_PORT", "PSCL_SHARE_GPU", "PSCL_DIST_BACKEND")}
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + os.environ.get("PYTHONPATH", "")
    if group:
        env.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    res = subprocess.run([sys.executable, *argv], cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert res.returncode == 0, (res.stdout + res.stderr)[-3000:]
    return res.stdout, res.stderr


def test_world1_rccl_group_equals_no_group(tmp_path):
    """The RCCL (backend nccl) collective path of every sharded entry point, executed on one GPU
    in a world-1 process group: run_fer_sweep --rng philox (counter all-reduce, max of the wall
    time), run_ber_sweep --rng philox at config 5's shape (all-gather + MIN/SUM all-reduces of the
    exact stop rule) and bench.py (timing MAX, counter SUM) give the same rows and counts as the
    same runs without a process group."""
    fer = ["-m", "polar_code_amd.eval.run_fer_sweep", "--M", "8", "--frames", "150000", "--snr_lo", "4.5",
           "--snr_hi", "5", "--snr_step", "0.5", "--retries", "8", "--beta", str(GOLDEN / "beta_M8.npy"),
           "--rng", "philox", "--batch", "60000", "--include_uncoded", "--no_plot"]
    ber = ["-m", "polar_code_amd.eval.run_ber_sweep", "--scheme", "nr_polar_scl", "--K_payload", "64", "--K_crc",
           "24", "--E", "256", "--N", "128", "--M", "8", "--EbN0_lo", "1.0", "--EbN0_hi", "2.0", "--EbN0_step",
           "0.5", "--bits_cap", "3000000", "--err_cap", "2000", "--rng", "philox", "--batch", "20000"]
    bench = ["bench.py", "--frames", "100000", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--extra", "none"]
    out = {}
    for group in (False, True):
        d = tmp_path / f"g{int(group)}"
        so, se = _world1(fer + ["--out_dir", str(d), "--plot_dir", str(d)], group)
        assert ("backend=nccl world=1" in se) == group, se[-2000:]
        fer_csv = (d / "fer_M8.csv").read_text()
        so, se = _world1(ber + ["--out", str(d / "ber.csv")], group)
        assert ("backend=nccl world=1" in se) == group, se[-2000:]
        ber_csv = (d / "ber.csv").read_text()
        so, _ = _world1(bench, group)
        line = json.loads([x for x in so.splitlines() if x.startswith("{")][-1])
        assert line["config"]["collective"] == ("nccl" if group else None)
        out[group] = (fer_csv, ber_csv, line["fer"])
    assert out[True][0] == out[False][0] and out[True][0].count("\n") == 3
    assert out[True][1] == out[False][1]
    assert out[True][2] == out[False][2] and out[True][2]["frames"] == 300_000


@pytest.mark.timeout(900)
def test_bench_gpus2_default_extras_equal_world1():
    """The driver's multi-GPU command with its default extras (`bench.py --gpus 2`, no --extra
    none): every extra config and the config-3 sweep run under a 2-rank process group (rank 0's
    oracle parity sample while the other rank waits at a collective included), rank 0's single
    line carries extra_configs and config3_sweep_L8, and every counter equals the world-1 run
    over the same global frames (world 1 decodes 2B frames per step, world 2 B per rank)."""
    B, S, E = 20_000, 2, 2
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(PSCL_SHARE_GPU="1", PSCL_DIST_BACKEND="gloo")
    line = {}
    for gpus, frames in ((1, 2 * B), (2, B)):
        cmd = [sys.executable, "bench.py", "--gpus", str(gpus), "--frames", str(frames), "--steps", str(S),
               "--warmup", "1", "--extra-steps", str(E), "--extra-parity", "4000", "--cpu-seconds", "1"]
        res = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
        assert res.returncode == 0, (res.stdout + res.stderr)[-3000:]
        lines = [x for x in res.stdout.splitlines() if x.startswith("{")]
        assert len(lines) == 1, res.stdout[-2000:]
        line[gpus] = json.loads(lines[0])
    w1, w2 = line[1], line[2]
    assert w2["n_gpus"] == 2 and w2["config"]["collective"] == "gloo"
    assert w2["cpu_baseline"] is None and w1["cpu_baseline"] is not None  # an N = 1 figure only
    assert w2["parity"]["mismatches"] == 0 and w1["parity"]["mismatches"] == 0
    assert w1["fer"]["frames"] == w2["fer"]["frames"] == 2 * B * S
    for k in ("frame_errors", "ber", "payload_fer", "payload_ber"):
        assert w1["fer"][k] == w2["fer"][k], k
    x1, x2 = w1["extra_configs"], w2["extra_configs"]
    assert set(x1) == set(x2) == {"config2_scl_L4", "config4_dlscl_L4_r8_beta4", "config5_nr_E256_L8",
                                  "config3_sweep_L8"}
    for name in ("config2_scl_L4", "config4_dlscl_L4_r8_beta4", "config5_nr_E256_L8"):
        assert x2[name]["fer"]["frames"] == x1[name]["fer"]["frames"] == 2 * B * E, name
        assert x2[name]["fer"]["frame_errors"] == x1[name]["fer"]["frame_errors"], name
        assert x2[name]["parity"]["mismatches"] == 0, name
        if "dl_scl" in x1[name]:
            assert x2[name]["dl_scl"]["frame_errors"] == x1[name]["dl_scl"]["frame_errors"], name
    s1, s2 = x1["config3_sweep_L8"], x2["config3_sweep_L8"]
    assert s1["frames_per_point"] == s2["frames_per_point"] == 2 * B
    assert [p["snr_db"] for p in s2["points"]] == [4.0, 4.5, 5.0, 5.5, 6.0, 6.5]
    for p1, p2 in zip(s1["points"], s2["points"]):
        for k in ("fer_scl", "fer_dl", "fer_uncoded", "avg_retries"):
            assert p1[k] == p2[k], (p1["snr_db"], k)
