"""Multi-process path on CPU (gloo, world_size 2): run_fer_sweep's frame sharding and its
counter all-reduce give the same CSV as one process.  The GPU decoder is replaced by the
oracle in the worker processes (test infrastructure), everything else is the product path."""
import multiprocessing as mp
import os
import socket
import sys
from pathlib import Path

import numpy as np

from polar_code_amd import dist

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_backends(mod):
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle

    def scl_batch(llr, info, M, crc, device):
        bits, ok = oracle.decode_batch(llr, info, M, crc)
        return {"best_bits": bits, "crc_pass": ok}

    def dl_batch(llr, info, M, retries, crc=None, beta=None, device=0, baseline=None):
        bits = baseline["best_bits"].copy()
        ok = baseline["crc_pass"].copy()
        att = np.ones(llr.shape[0], np.int32)
        for f in np.flatnonzero(~ok):
            r = oracle.decode_with_retries(llr[f], info, M, retries, crc=crc, beta=beta)
            bits[f], ok[f], att[f] = r["bits"], r["success"], r["attempts"]
        return {"best_bits": bits, "success": ok, "attempts": att}

    mod.scl_batch = scl_batch
    mod.dl_batch = dl_batch


def _worker(rank, world, port, out_dir, argv):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    from polar_code_amd.eval import run_fer_sweep as m

    _oracle_backends(m)
    m.dist.init(backend="gloo")
    m.run_sweep(m.build_argparser().parse_args(argv + ["--out_dir", out_dir, "--no_plot"]))
    m.dist.finalize()


def _run(world, out_dir, argv):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(out_dir), argv)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0


def test_shard_ranges_cover_exactly():
    for total in (0, 1, 7, 2000, 1000003):
        for world in (1, 2, 3, 8):
            ranges = [dist.shard(total, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            assert max(b - a for a, b in ranges) - min(b - a for a, b in ranges) <= 1


def test_two_rank_sweep_equals_one_rank(tmp_path):
    argv = ["--M", "4", "--frames", "601", "--snr_lo", "4.5", "--snr_hi", "5", "--snr_step", "0.5", "--retries", "8",
            "--beta", str(ROOT / "tests" / "golden" / "beta_M4.npy"), "--include_uncoded", "--batch", "128", "--dl_engine", "host"]
    (tmp_path / "w1").mkdir()
    (tmp_path / "w2").mkdir()
    _run(1, tmp_path / "w1", argv)
    _run(2, tmp_path / "w2", argv)
    a = (tmp_path / "w1" / "fer_M4.csv").read_text()
    b = (tmp_path / "w2" / "fer_M4.csv").read_text()
    assert a == b and a.count("\n") == 3
