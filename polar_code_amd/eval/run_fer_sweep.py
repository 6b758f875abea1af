"""FER sweep: SCL vs DL-SCL (mirror of dl_scl_polar/eval/run_fer_sweep.py, same flags,
console lines, CSV schema and plot).

    python -m polar_code_amd.eval.run_fer_sweep --M 8 --frames 2000 --snr_lo 5 --snr_hi 5 \
        --snr_step 0 --retries 8 --beta tests/golden/beta_M8.npy --seed 0 --include_uncoded

Every decode runs on the GPU (libpolar_mi355x.so); by default the DL-SCL retry loop too
(--dl_engine device; --dl_engine host ranks flips with the reference's numpy calls).
Two channel modes:
  --rng replay  (default) the reference's own NumPy PCG64 stream, frame by frame in its draw
                order (run_fer_sweep.py:61,79-87,111-113): reproduces results/fer_M{4,8}.csv
                exactly.  Frames are generated on the host and decoded in batches.
  --rng philox  frames generated on the GPU by a counter-based Philox stream keyed by
                (seed, SNR, global frame index): results independent of GPU count,
                statistically equivalent to the reference (same channel model).
Multi-GPU: launch with torchrun; frames are sharded by global index and the counters are
summed with one all-reduce per SNR point (polar_code_amd/dist.py).
"""
from __future__ import annotations

import argparse
import math
import os
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Dict, List, Tuple

import numpy as np

from .. import _native, config, dist
from ..dlscl.flip import decode_with_retries, decode_with_retries_batch, decode_with_retries_device, words_to_bits
from ..polar.crc import attach_crc
from ..polar.polar import construct_info_set, encode
from ..polar.scl import decode_scl
from ..utils.seeding import philox_stream_id, seed_all

# counter vector, summed across ranks
C_FRAMES, C_SCL_ERR, C_DL_ERR, C_SCL_BIT, C_DL_BIT, C_UNC_ERR, C_UNC_BIT, C_BITS, C_BITS_UNC, C_DL_WORK = range(10)
NCOUNT = 10


def _bpsk(bits: np.ndarray) -> np.ndarray:
    return 1.0 - 2.0 * bits


def simulate_frame(llr, info_set, M, crc_poly, retries, beta) -> Tuple[Dict, Dict]:
    """Baseline SCL and DL-SCL of one frame (run_fer_sweep.py:28-38)."""
    base = decode_scl(llr, info_set, M, crc=crc_poly)
    dl = decode_with_retries(llr, info_set, M, retries, crc=crc_poly, beta=beta)
    return base, dl


def noise_params(snr_db: float, rate: float) -> Tuple[float, float, float, float]:
    ebno = 10 ** (snr_db / 10.0)
    var_c = 1.0 / (2.0 * rate * ebno)
    var_u = 1.0 / (2.0 * ebno)
    return var_c, math.sqrt(var_c), var_u, math.sqrt(var_u)


class ReplayStream:
    """The reference's per-SNR stream default_rng(seed + int(snr*10)) (run_fer_sweep.py:61),
    drawn in its order per frame: integers(0,2,payload) -> normal(0,sigma,N) ->
    [normal(0,sigma_u,payload)] (:79-87, :111-113).  One generator per sweep point, advanced
    block by block: frames [start, stop) cost O(stop - position) draws, so a whole point costs
    O(frames) (a rank of a sharded run still draws past the frames of the ranks before it:
    ziggurat normals consume a variable number of words, the stream cannot jump)."""

    def __init__(self, seed: int, snr_db: float, payload_bits: int, crc_poly: str, include_uncoded: bool):
        cfg = config.get_config()
        self.N = cfg.N
        self.seed, self.snr_db = seed, snr_db
        self.payload_bits, self.crc_poly, self.include_uncoded = payload_bits, crc_poly, include_uncoded
        self.var_c, self.sig_c, self.var_u, self.sig_u = noise_params(snr_db, cfg.K / cfg.N)
        self._restart()

    def _restart(self) -> None:
        self.rng = np.random.default_rng(self.seed + int(self.snr_db * 10))
        self.pos = 0

    def _draw(self):
        p = self.rng.integers(0, 2, size=self.payload_bits, dtype=np.int8)
        z = self.rng.normal(0.0, self.sig_c, size=self.N)
        zu = self.rng.normal(0.0, self.sig_u, size=self.payload_bits) if self.include_uncoded else None
        self.pos += 1
        return p, z, zu

    def take(self, start: int, stop: int):
        """(payload, msg, llr, llr_unc) of frames [start, stop); blocks in increasing order
        continue the stream, an earlier start restarts it."""
        if start < self.pos:
            self._restart()
        while self.pos < start:
            self._draw()
        n = stop - start
        payload = np.empty((n, self.payload_bits), np.int8)
        noise = np.empty((n, self.N))
        unc = np.empty((n, self.payload_bits)) if self.include_uncoded else None
        for i in range(n):
            payload[i], noise[i], zu = self._draw()
            if self.include_uncoded:
                unc[i] = zu
        msg = attach_crc(payload, self.crc_poly)
        llr = 2.0 * (_bpsk(encode(msg)) + noise) / self.var_c
        llr_unc = 2.0 * (_bpsk(payload) + unc) / self.var_u if self.include_uncoded else None
        return payload, msg, llr, llr_unc


def replay_stream(seed: int, snr_db: float, start: int, stop: int, payload_bits: int, crc_poly: str,
                  include_uncoded: bool):
    """Frames [start, stop) of the reference's per-SNR stream (a fresh ReplayStream)."""
    return ReplayStream(seed, snr_db, payload_bits, crc_poly, include_uncoded).take(start, stop)


def scl_batch(llr, info_set, M, crc, device):
    """Batched decode_scl on the GPU: best_path_bits [B, K] and CRC pass [B]."""
    dec = _native.get_decoder(llr.shape[1], info_set, M, crc, device)
    return dec.decode(llr, want_metrics=False, want_cands=False, want_info_llrs=False)


dl_batch = decode_with_retries_batch


def _count_block(c, msg, llr, payload, llr_unc, info_set, M, crc, retries, beta, device, engine="device"):
    if engine == "device":  # SCL + the whole DL-SCL retry loop on the GPU
        out = decode_with_retries_device(llr, info_set, M, retries, crc=crc, beta=beta, device=device, msg=msg)
        cs, cd = out["counters"]["scl"], out["counters"]["dl"]
        c[C_FRAMES] += llr.shape[0]
        c[C_SCL_ERR] += int(cs[_native.CNT_FRAME_ERR])
        c[C_SCL_BIT] += int(cs[_native.CNT_BIT_ERR])
        c[C_DL_ERR] += int(cd[_native.CNT_FRAME_ERR])
        c[C_DL_BIT] += int(cd[_native.CNT_BIT_ERR])
        c[C_DL_WORK] += int(cd[_native.CNT_RETRIES])
    else:  # GPU decodes, flip ranking with the reference's numpy calls on the host
        base = scl_batch(llr, info_set, M, crc, device)
        c[C_FRAMES] += llr.shape[0]
        c[C_SCL_ERR] += int(np.count_nonzero(~base["crc_pass"]))
        c[C_SCL_BIT] += int(np.count_nonzero(base["best_bits"] != msg))
        dl = dl_batch(llr, info_set, M, retries, crc=crc, beta=beta, device=device, baseline=base)
        c[C_DL_ERR] += int(np.count_nonzero(~dl["success"]))
        c[C_DL_BIT] += int(np.count_nonzero(dl["best_bits"] != msg))
        c[C_DL_WORK] += int((dl["attempts"] - 1).sum())
    c[C_BITS] += msg.size
    if llr_unc is not None:
        errs = np.count_nonzero((llr_unc < 0).astype(np.int8) != payload, axis=1)
        c[C_UNC_ERR] += int(np.count_nonzero(errs))
        c[C_UNC_BIT] += int(errs.sum())
        c[C_BITS_UNC] += payload.size


class _SweepBuffers:
    """Device buffers of one Philox batch shape, kept across batches and SNR points."""

    def __init__(self, dec, n: int):
        self.dec, self.n = dec, n
        N = dec.N
        self.mem = _native.DeviceArena(dec)
        self.llr = self.mem.alloc(n * N * 8)
        self.msg = self.mem.alloc(n * dec.W * 8)
        self.best = self.mem.alloc(n * dec.W * 8)
        self.flags = self.mem.alloc(n)
        self.cnt = self.mem.alloc(3 * _native.PSCL_NCOUNT * 8)  # SCL, DL-SCL, uncoded

    def close(self):
        self.mem.__exit__(None, None, None)


_BUFS: Dict = {}


def _buffers(dec, n: int) -> _SweepBuffers:
    """One buffer set per handle, reallocated when the batch size grows."""
    buf = _BUFS.get(id(dec))
    if buf is None or buf.n < n:
        if buf is not None:
            buf.close()
        buf = _BUFS[id(dec)] = _SweepBuffers(dec, n)
    return buf


def _add_common(c, cs, cu, n, K, payload_bits, include_uncoded):
    c[C_FRAMES] += n
    c[C_SCL_ERR] += int(cs[_native.CNT_FRAME_ERR])
    c[C_SCL_BIT] += int(cs[_native.CNT_BIT_ERR])
    c[C_BITS] += n * K
    if include_uncoded:
        c[C_UNC_ERR] += int(cu[_native.CNT_FRAME_ERR])
        c[C_UNC_BIT] += int(cu[_native.CNT_BIT_ERR])
        c[C_BITS_UNC] += n * payload_bits


def _philox_sweep_device(args, snr_points, ranges, info_set, beta, device, payload_bits):
    """Every SNR point of this rank on the device in ONE pipelined pass: per block one
    pscl_simulate_device call (TX, uncoded baseline, SCL + DL-SCL, counters added on the device),
    the handle pipelined so each block's DL-SCL retry chains overlap the next block's -- and the
    next SNR point's -- TX and baseline decode; one join at the end.  Returns int64 counters
    [points, 3, PSCL_NCOUNT] (rows SCL, DL-SCL, uncoded), equal to per-point pscl_simulate calls."""
    cfg = config.get_config()
    dec = _native.get_decoder(cfg.N, info_set, args.M, cfg.crc_poly, device)
    dec.set_beta(beta)
    nc = _native.PSCL_NCOUNT
    batch = args.batch or (1 << 20)
    dec.set_pipelined(True)
    try:
        with _native.DeviceArena(dec) as mem:
            d_cnt = mem.alloc(len(snr_points) * 3 * nc * 8)
            mem.memset(d_cnt, 0, len(snr_points) * 3 * nc * 8)
            for i, snr_db in enumerate(snr_points):
                start, stop = ranges[i]
                for b0 in range(start, stop, batch):
                    dec.simulate_device(args.seed, philox_stream_id(float(snr_db)), float(snr_db), cfg.K / cfg.N,
                                        payload_bits, b0, min(stop, b0 + batch) - b0, args.retries,
                                        args.include_uncoded, d_cnt + i * 3 * nc * 8)
            dec.join()
            dec.sync()
            return mem.download(d_cnt, len(snr_points) * 3 * nc * 8, np.int64).reshape(len(snr_points), 3, nc)
    finally:
        dec.set_pipelined(False)


def _philox_block(c, seed, snr_db, frame0, n, info_set, M, crc, retries, beta, device, include_uncoded,
                  payload_bits, engine="device", slot=0):
    """n frames generated on the device; SCL, DL-SCL and the uncoded baseline counted there."""
    cfg = config.get_config()
    dec = _native.get_decoder(cfg.N, info_set, M, crc, device, slot=slot)
    sid = philox_stream_id(snr_db)
    if engine == "device":  # TX, uncoded baseline, SCL + DL-SCL and counting: one library call
        dec.set_beta(beta)
        cs, cd, cu = dec.simulate(seed, sid, snr_db, cfg.K / cfg.N, payload_bits, frame0, n, retries, include_uncoded)
        c[C_DL_ERR] += int(cd[_native.CNT_FRAME_ERR])
        c[C_DL_BIT] += int(cd[_native.CNT_BIT_ERR])
        c[C_DL_WORK] += int(cd[_native.CNT_RETRIES])
        _add_common(c, cs, cu, n, cfg.K, payload_bits, include_uncoded)
        return
    # host engine: the GPU decodes and counts the baseline, flips are ranked with numpy
    W = dec.W
    buf = _buffers(dec, n)
    mem = buf.mem
    nc = _native.PSCL_NCOUNT
    d_cs, d_cu = buf.cnt, buf.cnt + 2 * nc * 8
    mem.memset(buf.cnt, 0, 3 * nc * 8)
    dec.channel_device(seed, sid, snr_db, cfg.K / cfg.N, payload_bits, frame0, n, buf.llr, buf.msg)
    if include_uncoded:
        dec.uncoded_device(seed, sid, snr_db, payload_bits, frame0, n, d_cu)
    dec.decode_device(buf.llr, n, d_best=buf.best, d_flags=buf.flags, d_ref=buf.msg, k_payload=payload_bits,
                      d_counters=d_cs)
    cs, _, cu = mem.download(buf.cnt, 3 * nc * 8, np.int64).reshape(3, nc)
    flags = mem.download(buf.flags, n, np.uint8)
    fail = np.flatnonzero((flags & _native.PSCL_FLAG_CRC_PASS) == 0)
    dl_bit = int(cs[_native.CNT_BIT_ERR])
    if fail.size and retries > 0:
        llr_all = mem.download(buf.llr, n * cfg.N * 8, np.float64).reshape(n, cfg.N)
        msg_f = words_to_bits(mem.download(buf.msg, n * W * 8, np.uint64).reshape(n, W)[fail], cfg.K)
        base_f = words_to_bits(mem.download(buf.best, n * W * 8, np.uint64).reshape(n, W)[fail], cfg.K)
        dl = decode_with_retries_batch(llr_all[fail], info_set, M, retries, crc=crc, beta=beta, device=device,
                                       baseline={"best_bits": base_f, "crc_pass": np.zeros(fail.size, bool)})
        c[C_DL_ERR] += int(np.count_nonzero(~dl["success"]))
        dl_bit += int(np.count_nonzero(dl["best_bits"] != msg_f)) - int(np.count_nonzero(base_f != msg_f))
        c[C_DL_WORK] += int((dl["attempts"] - 1).sum())
    else:
        c[C_DL_ERR] += int(fail.size)
    c[C_DL_BIT] += dl_bit
    _add_common(c, cs, cu, n, cfg.K, payload_bits, include_uncoded)


_BETA_CACHE: Dict[tuple, np.ndarray] = {}


def _load_beta(path) -> np.ndarray:
    """np.load of a beta checkpoint, cached by (path, size, mtime): a sweep service re-running
    run_sweep on the same checkpoint skips the file read (~0.1-0.2 ms per sweep)."""
    st = os.stat(path)
    key = (os.path.abspath(path), st.st_size, st.st_mtime_ns)
    b = _BETA_CACHE.get(key)
    if b is None:
        if len(_BETA_CACHE) > 16:
            _BETA_CACHE.clear()
        b = _BETA_CACHE[key] = np.load(path)
        b.setflags(write=False)
    return b


def run_sweep(args: argparse.Namespace) -> List[Dict[str, float]]:
    cfg = config.get_config()
    seed_all(args.seed)
    ctx = dist.init()
    device = ctx.device
    engine = args.dl_engine
    if args.device == "cpu":  # the product's host decoder (pscl_decode_cpu), no GPU touched
        if args.rng != "replay":
            raise ValueError("--device cpu decodes the reference's NumPy stream (--rng replay); philox is on-device")
        device, engine = "cpu", "host"
    info_set = construct_info_set(cfg.N, cfg.K)
    payload_bits = cfg.K - cfg.crc_bits
    snr_points = (np.arange(args.snr_lo, args.snr_hi + 1e-9, args.snr_step) if args.snr_step > 0
                  else np.array([args.snr_lo]))
    beta = _load_beta(args.beta) if args.beta else None
    results: List[Dict[str, float]] = []
    t0 = time.perf_counter()
    # philox + device engine: the whole sweep enqueued at once (retry chains overlap the next
    # point's TX and baseline), the counters read at the end
    sweep_cnt = None
    if args.rng == "philox" and engine == "device":
        rng_ = [dist.shard(args.frames, ctx.rank, ctx.world)] * len(snr_points)
        sweep_cnt = _philox_sweep_device(args, snr_points, rng_, info_set, beta, device, payload_bits)
    for ip, snr_db in enumerate(snr_points):
        c = np.zeros(NCOUNT, np.int64)
        start, stop = dist.shard(args.frames, ctx.rank, ctx.world)
        # philox: one pscl_simulate call per 2^20 frames by default -- a call's DL-SCL retry rounds
        # are latency-bound at high SNR (few entries, 8 rounds), so fewer, larger calls win
        # (5 dB, 10^6 frames: 155 M frames/s at 2^19 on two streams, 185 M at 2^20)
        batch = args.batch or (1 << 20 if args.rng == "philox" else 1 << 19)
        blocks = [(b0, min(stop, b0 + batch)) for b0 in range(start, stop, batch)]
        if sweep_cnt is not None:
            cs, cd, cu = sweep_cnt[ip]
            c[C_DL_ERR] += int(cd[_native.CNT_FRAME_ERR])
            c[C_DL_BIT] += int(cd[_native.CNT_BIT_ERR])
            c[C_DL_WORK] += int(cd[_native.CNT_RETRIES])
            _add_common(c, cs, cu, stop - start, cfg.K, payload_bits, args.include_uncoded)
        elif args.rng == "replay":
            stream = ReplayStream(args.seed, float(snr_db), payload_bits, cfg.crc_poly, args.include_uncoded)
            for b0, b1 in blocks:
                payload, msg, llr, llr_unc = stream.take(b0, b1)
                _count_block(c, msg, llr, payload, llr_unc, info_set, args.M, cfg.crc_poly, args.retries, beta, device,
                             engine)
        else:
            # batches in flight on `--streams` handles (own HIP streams), one host thread each:
            # one batch's TX and DL-SCL retry chain overlap another's decode; counts add exactly
            def work(slot):
                cs = np.zeros(NCOUNT, np.int64)
                for b0, b1 in blocks[slot::nstreams]:
                    _philox_block(cs, args.seed, float(snr_db), b0, b1 - b0, info_set, args.M, cfg.crc_poly,
                                  args.retries, beta, device, args.include_uncoded, payload_bits, engine, slot)
                return cs
            nstreams = max(1, min(args.streams, len(blocks)))
            if nstreams == 1:
                c += work(0)
            else:
                with ThreadPoolExecutor(nstreams) as ex:
                    for cs in ex.map(work, range(nstreams)):
                        c += cs
        c = dist.allreduce_sum(c, ctx)
        total_frames = args.frames
        scl_fer = c[C_SCL_ERR] / total_frames
        dl_fer = c[C_DL_ERR] / total_frames
        row = {"snr_db": float(snr_db), "fer_scl": scl_fer, "fer_dl": dl_fer}
        row["ber_scl"] = c[C_SCL_BIT] / c[C_BITS] if c[C_BITS] > 0 else float("nan")
        row["ber_dl"] = c[C_DL_BIT] / c[C_BITS] if c[C_BITS] > 0 else float("nan")
        row["avg_retries"] = c[C_DL_WORK] / max(total_frames, 1)
        if args.include_uncoded:
            row["fer_uncoded"] = c[C_UNC_ERR] / total_frames if total_frames > 0 else float("nan")
            row["ber_uncoded"] = c[C_UNC_BIT] / c[C_BITS_UNC] if c[C_BITS_UNC] > 0 else float("nan")
            msg_line = (f"SNR={snr_db:.2f} dB -> Uncoded FER={row['fer_uncoded']:.3e}, BER={row['ber_uncoded']:.3e}; "
                        f"SCL FER={scl_fer:.3e}, BER={row['ber_scl']:.3e}; DL FER={dl_fer:.3e}, BER={row['ber_dl']:.3e}")
        else:
            msg_line = (f"SNR={snr_db:.2f} dB -> SCL FER={scl_fer:.3e}, BER={row['ber_scl']:.3e}; "
                        f"DL FER={dl_fer:.3e}, BER={row['ber_dl']:.3e}")
        if ctx.is_root:
            print(msg_line, flush=True)
        results.append(row)
    elapsed = dist.allreduce_max(time.perf_counter() - t0, ctx)
    if ctx.is_root:
        write_outputs(results, args)
        if args.verbose:
            where = "the host CPU" if device == "cpu" else f"{ctx.world} GPU(s)"
            print(f"decoded {args.frames * len(snr_points)} frames x2 (SCL + DL-SCL) on {where} in "
                  f"{elapsed:.2f} s ({args.rng} channel)")
    return results


def write_outputs(results: List[Dict[str, float]], args: argparse.Namespace) -> None:
    """CSV (run_fer_sweep.py:150-173) and semilogy plot (:175-191)."""
    output_dir = Path(args.out_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    csv_path = output_dir / f"fer_M{args.M}.csv"
    with csv_path.open("w") as f:
        headers = ["snr_db"]
        if args.include_uncoded:
            headers.extend(["fer_uncoded", "ber_uncoded"])
        headers.extend(["fer_scl", "ber_scl", "fer_dl", "ber_dl"])
        f.write(",".join(headers) + "\n")
        for row in results:
            values = [f"{row['snr_db']:.3f}"]
            if args.include_uncoded:
                values.extend([f"{row['fer_uncoded']:.6e}", f"{row['ber_uncoded']:.6e}"])
            values.extend([f"{row['fer_scl']:.6e}", f"{row['ber_scl']:.6e}", f"{row['fer_dl']:.6e}",
                           f"{row['ber_dl']:.6e}"])
            f.write(",".join(values) + "\n")
    print(f"Saved FER table to {csv_path}")
    if args.no_plot:
        return
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        print("matplotlib not available; skipping plot")
        return
    plot_dir = Path(args.plot_dir)
    plot_dir.mkdir(parents=True, exist_ok=True)
    plot_path = plot_dir / f"fer_M{args.M}.png"
    plt.figure(figsize=(6, 4))
    snrs = [row["snr_db"] for row in results]
    if args.include_uncoded:
        plt.semilogy(snrs, [row["fer_uncoded"] for row in results], "^-", label="Uncoded")
    plt.semilogy(snrs, [row["fer_scl"] for row in results], "o-", label="SCL")
    plt.semilogy(snrs, [row["fer_dl"] for row in results], "s-", label="DL-SCL")
    plt.xlabel("Eb/N0 (dB)")
    plt.ylabel("Frame Error Rate")
    plt.grid(True, which="both", ls="--", alpha=0.4)
    plt.legend()
    plt.tight_layout()
    plt.savefig(plot_path, dpi=200)
    plt.close()
    print(f"Saved FER plot to {plot_path}")


def build_argparser() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser(description="Run FER sweep for DL-SCL")
    parser.add_argument("--M", type=int, required=True, help="List size")
    parser.add_argument("--frames", type=int, default=10000, help="Frames per SNR point")
    parser.add_argument("--snr_lo", type=float, default=4.0)
    parser.add_argument("--snr_hi", type=float, default=6.5)
    parser.add_argument("--snr_step", type=float, default=0.5)
    parser.add_argument("--retries", type=int, default=8)
    parser.add_argument("--beta", type=str, help="Path to trained beta matrix (.npy)")
    parser.add_argument("--seed", type=int, default=0)
    parser.add_argument("--out_dir", type=str, default="results")
    parser.add_argument("--plot_dir", type=str, default="plots")
    parser.add_argument("--include_uncoded", action="store_true", help="Also simulate an uncoded BPSK baseline")
    # engine options (not in the reference)
    parser.add_argument("--rng", choices=["replay", "philox"], default="replay",
                        help="replay: reference NumPy stream (exact); philox: on-device generation")
    parser.add_argument("--batch", type=int, default=None,
                        help="frames per GPU batch (default 2^20 with --rng philox, 2^19 with replay)")
    parser.add_argument("--streams", type=int, default=2,
                        help="philox: batches in flight per GPU (one handle/stream and host thread each)")
    parser.add_argument("--dl_engine", choices=["device", "host"], default="device",
                        help="device: DL-SCL retry loop on the GPU; host: numpy flip ranking (reference calls)")
    parser.add_argument("--device", choices=["gpu", "cpu"], default="gpu",
                        help="cpu: the product's host decoder (no GPU; --rng replay, host flip ranking)")
    parser.add_argument("--no_plot", action="store_true")
    parser.add_argument("--verbose", action="store_true")
    return parser


def main(argv: List[str] | None = None) -> None:
    args = build_argparser().parse_args(argv)
    run_sweep(args)
    dist.finalize()


if __name__ == "__main__":
    main()
