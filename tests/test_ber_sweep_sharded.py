"""run_ber_sweep --rng philox on CPU: the sharded stop rule (gloo, world 1..3).

The frame source (PhiloxFrames: device TX + decode) is replaced by a deterministic function of
the global frame index (test infrastructure); everything else -- round sizing, per-rank
contiguous ranges, the all-gather of partial sums, the exact first global frame meeting
`bit_errors >= err_cap or bits_total >= bits_cap` (run_ber_sweep.py:127), the MIN/SUM
all-reduces and the rows -- is the product code.  Rows must equal a frame-by-frame sequential
scan of the same per-frame errors, whatever the world size and batch size."""
import multiprocessing as mp
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

from polar_code_amd.eval import run_ber_sweep as rb

ROOT = Path(__file__).resolve().parent.parent


class FakeFrames:
    """Per-frame payload bit errors and work as a fixed function of (SNR, global frame)."""

    def __init__(self, payload_len):
        self.payload_len = payload_len

    def frames(self, seed, EbN0_dB, frame0, n):
        g = np.arange(frame0, frame0 + n, dtype=np.int64)
        x = (g * 2654435761 + int(round(EbN0_dB * 10)) * 40503 + seed * 977) % 1000
        thresh = int(300 * 0.25 ** EbN0_dB)  # fewer error frames at higher SNR
        err = np.where(x < thresh, x % 7 + 1, 0).astype(np.int64)
        return err, (x % 3).astype(np.float64)


def sequential_row(src, EbN0_dB, args, payload_len):
    """The reference's loop, frame by frame (run_ber_sweep.py:127-169)."""
    st = rb.SimulationStats()
    g = 0
    while st.bit_errors < args.err_cap and st.bits_total < args.bits_cap:
        e, w = src.frames(args.seed, EbN0_dB, g, 1)
        st.update(int(e[0]), float(w[0]), bool(e[0] > 0), payload_len)
        g += 1
    return st.row()


def _args(batch, err_cap=300, bits_cap=2e5):
    return rb.parse_args(["--scheme", "polar_scl", "--K_payload", "40", "--K_crc", "24", "--E", "128",
                          "--EbN0_lo", "1", "--EbN0_hi", "4", "--EbN0_step", "1", "--err_cap", str(err_cap),
                          "--bits_cap", str(bits_cap), "--out", "x.csv", "--batch", str(batch), "--rng", "philox"])


def _rows(args, ctx=None):
    src = FakeFrames(40)
    return [rb.run_scheme_philox(src, float(s), args, 128, 40, "M=4", ctx) for s in (1.0, 2.0, 3.0, 4.0)]


@pytest.mark.parametrize("batch", [1, 7, 64, 5000])
def test_single_rank_stop_equals_sequential(batch):
    args = _args(batch)
    src = FakeFrames(40)
    for row, s in zip(_rows(args), (1.0, 2.0, 3.0, 4.0)):
        ref = sequential_row(src, s, args, 40)
        for k in ("bits_total", "bit_errors", "ber", "fer", "avg_work"):
            assert row[k] == ref[k], (s, k, row[k], ref[k])
    # both stop rules occur in this grid
    rows = _rows(args)
    assert any(r["bit_errors"] >= 300 for r in rows) and any(r["bits_total"] >= 2e5 for r in rows)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, batch, out):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    from polar_code_amd import dist
    from polar_code_amd.eval import run_ber_sweep as m

    ctx = dist.init(backend="gloo")
    args = _args(batch)
    src = FakeFrames(40)
    rows = [m.run_scheme_philox(src, float(s), args, 128, 40, "M=4", ctx) for s in (1.0, 2.0, 3.0, 4.0)]
    if rank == 0:
        m.write_csv(rows, Path(out))
    dist.finalize()


def _run(world, batch, out):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, str(out))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0


def test_sharded_rows_equal_single_rank(tmp_path):
    ref = tmp_path / "ref.csv"
    rb.write_csv(_rows(_args(64)), ref)
    for world, batch in ((2, 64), (3, 13)):
        out = tmp_path / f"w{world}.csv"
        _run(world, batch, out)
        assert out.read_text() == ref.read_text(), world


def test_payload_errors_from_words():
    rng = np.random.default_rng(3)
    for K, kp in ((64, 40), (88, 64), (88, 70), (130, 100)):
        W = (K + 63) // 64
        a = rng.integers(0, 2, size=(50, K), dtype=np.int8)
        b = a.copy()
        flip = rng.random((50, K)) < 0.1
        b[flip] ^= 1

        def words(x):
            w = np.zeros((x.shape[0], W), np.uint64)
            for j in range(K):
                w[:, j >> 6] |= x[:, j].astype(np.uint64) << np.uint64(j & 63)
            return w

        got = rb.payload_errors_from_words(words(a), words(b), kp)
        np.testing.assert_array_equal(got, np.count_nonzero(a[:, :kp] != b[:, :kp], axis=1))


def test_replay_refuses_multi_rank(monkeypatch):
    from polar_code_amd import dist

    monkeypatch.setattr(dist, "init", lambda backend=None: dist.Context(rank=0, world=2))
    args = rb.parse_args(["--scheme", "polar_scl", "--K_payload", "8", "--K_crc", "0", "--E", "16", "--EbN0_lo", "5",
                          "--EbN0_hi", "5", "--out", "x.csv"])
    with pytest.raises(ValueError, match="philox"):
        rb.run(args)
