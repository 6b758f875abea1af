"""BER/FER sweeps across schemes (mirror of dl_scl_polar/eval/run_ber_sweep.py: same flags,
rows and CSV).  Schemes polar_scl, dl_scl and nr_polar_scl decode on the GPU; nr_ldpc (the
reference's 3x6 demo base graph) is out of scope.

The reference draws every frame from ONE NumPy stream shared by all SNR points
(run_ber_sweep.py:230) and stops each point on a data-dependent rule
(`while bit_errors < err_cap and bits_total < bits_cap`, :127).  Two channel modes:

  --rng replay  (default) frames generated in batches from that same stream and decoded in one
                GPU call; the exact stop frame is found with a prefix sum, and if a batch
                overshoots, the stream is rewound to the batch start and advanced by exactly
                the frames the reference would have drawn -- so the rows (and the stream handed
                to the next SNR point) are identical to the reference's.  One process.
  --rng philox  frames generated on the GPU (pscl_channel_device: payload -> CRC -> polar
                encode [-> NR interleave/repeat] -> BPSK -> AWGN -> LLR), keyed by (seed, SNR,
                global frame index), so the rows do not depend on the number of GPUs.  Under
                torchrun each round of world x --batch frames is split into contiguous global
                ranges per rank; one all-gather of per-rank partial sums per round, and in the
                round where the stop rule fires, the first global frame with
                bit_errors >= err_cap or bits_total >= bits_cap is found exactly (each rank scans
                its own range from the prefix of the ranks before it; one MIN and one SUM
                all-reduce), so a sharded sweep writes the same rows as one GPU.
"""
from __future__ import annotations

import argparse
import math
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, Iterable, List, Optional

import numpy as np

from .. import _native, dist
from .. import config as global_config
from ..dlscl.flip import decode_with_retries_batch
from ..nr.polar.interleaver import subblock_interleave
from ..polar import polar as polar_core
from ..polar.crc import attach_crc
from ..polar.polar import construct_info_set
from ..utils.seeding import philox_stream_id, seed_all


@dataclass
class SimulationStats:
    bits_total: int = 0
    bit_errors: int = 0
    frame_errors: int = 0
    work_sum: float = 0.0
    frames: int = 0

    def update(self, bit_err: int, work: float, frame_error: bool, payload_len: int) -> None:
        self.bits_total += payload_len
        self.bit_errors += bit_err
        self.work_sum += work
        self.frames += 1
        if frame_error:
            self.frame_errors += 1

    def row(self) -> Dict[str, float]:
        ber = self.bit_errors / self.bits_total if self.bits_total > 0 else float("nan")
        fer = self.frame_errors / self.frames if self.frames > 0 else float("nan")
        avg_work = self.work_sum / self.frames if self.frames > 0 else 0.0
        return {"bits_total": self.bits_total, "bit_errors": self.bit_errors, "ber": ber, "fer": fer,
                "avg_work": avg_work}


def _polar_encode(info_bits: np.ndarray, info_set: np.ndarray, N: int) -> np.ndarray:
    """u[info_set] = info_bits; x = u G_N (run_ber_sweep.py:65-70); batch-capable."""
    info_bits = np.asarray(info_bits)
    if info_bits.shape[-1] != info_set.size:
        raise ValueError("info_bits length must match info_set size")
    u = np.zeros(info_bits.shape[:-1] + (N,), dtype=np.int8)
    u[..., info_set] = info_bits
    return polar_core._polar_transform(u)


def _bpsk(bits: np.ndarray) -> np.ndarray:
    return 1.0 - 2.0 * bits.astype(np.float64)


def _payload_bit_errors(payload: np.ndarray, candidate: Optional[np.ndarray], K_payload: int) -> int:
    if candidate is None:
        return int(K_payload)
    if candidate.size < K_payload:
        raise ValueError("Candidate bits shorter than payload")
    return int(np.count_nonzero(payload != candidate[:K_payload]))


def _noise_params(EbN0_dB: float, payload_bits: int, coded_bits: int) -> float:
    ebno_lin = 10 ** (EbN0_dB / 10.0)
    rate = payload_bits / coded_bits
    esn0_lin = ebno_lin * rate
    return 1.0 / (2.0 * esn0_lin)


class _Scheme:
    """Batched encoder + GPU decoder for one scheme."""

    def __init__(self, args, info_set, N):
        self.args, self.info_set, self.N = args, info_set, N
        self.beta = np.load(args.beta) if (args.scheme == "dl_scl" and args.beta) else None

    def encode(self, payload: np.ndarray) -> np.ndarray:
        a = self.args
        if a.scheme in ("polar_scl", "dl_scl"):
            info_bits = payload if a.K_crc == 0 else attach_crc(payload, a.crc_poly)
            return _polar_encode(info_bits, self.info_set, self.N)
        # nr_polar_scl: encode_rate_matched per frame (scl_nr.py:23-35), vectorised
        msg = attach_crc(payload[..., : a.K_payload], a.crc_poly)
        code = _polar_encode(msg, self.info_set, self.N)
        ilv = np.stack([subblock_interleave(c) for c in code]) if code.ndim == 2 else subblock_interleave(code)
        if a.E <= ilv.shape[-1]:
            return ilv[..., : a.E]
        reps = -(-a.E // ilv.shape[-1])
        return np.concatenate([ilv] * reps, axis=-1)[..., : a.E]

    def decode(self, llr: np.ndarray):
        """Returns (candidate bits [B, K_total], work [B])."""
        a = self.args
        B = llr.shape[0]
        crc = a.crc_poly if a.K_crc else None
        if a.scheme == "polar_scl":
            dec = _native.get_decoder(self.N, self.info_set, a.M, crc, a.device)
            out = dec.decode(llr, want_metrics=False, want_cands=False, want_info_llrs=False)
            return out["best_bits"], np.zeros(B)
        if a.scheme == "dl_scl":
            out = decode_with_retries_batch(llr, self.info_set, a.M, a.retries, crc=crc, beta=self.beta,
                                            device=a.device)
            return out["best_bits"], (out["attempts"] - 1).astype(float)
        dec = _native.get_decoder(self.N, self.info_set, a.M, a.crc_poly, a.device, E=a.E)
        out = dec.decode(llr, want_metrics=False, want_cands=False, want_info_llrs=False)
        return out["best_bits"], np.zeros(B)


def run_scheme(rng, EbN0_dB, args, info_set, scheme: _Scheme, coded_len, payload_len, params_label) -> Dict:
    """One SNR point (run_ber_sweep.py:112-181), batched with an exact stop."""
    stats = SimulationStats()
    noise_var = _noise_params(EbN0_dB, payload_len, coded_len)
    noise_sigma = math.sqrt(noise_var)
    sym_len = scheme.encode(np.zeros(payload_len, np.int8)).shape[-1]  # symbols per frame
    while stats.bit_errors < args.err_cap and stats.bits_total < args.bits_cap:
        left = max(1, math.ceil((args.bits_cap - stats.bits_total) / payload_len))
        B = int(min(args.batch or 4096, left))
        state = rng.bit_generator.state
        payload = np.empty((B, payload_len), np.int8)
        noise = np.empty((B, sym_len))
        for f in range(B):  # the reference's per-frame draw order (run_ber_sweep.py:128,140)
            payload[f] = rng.integers(0, 2, size=payload_len, dtype=np.int8)
            noise[f] = rng.normal(0.0, noise_sigma, size=sym_len)
        codeword = scheme.encode(payload)
        llr = 2.0 * (_bpsk(codeword) + noise) / noise_var
        cand, work = scheme.decode(llr)
        bit_err = np.count_nonzero(payload != cand[:, :payload_len], axis=1)
        cum_err = stats.bit_errors + np.cumsum(bit_err)
        cum_bits = stats.bits_total + payload_len * np.arange(1, B + 1)
        stop = np.flatnonzero((cum_err >= args.err_cap) | (cum_bits >= args.bits_cap))
        used = int(stop[0]) + 1 if stop.size else B
        if used < B:  # rewind: the reference draws exactly `used` frames at this point
            rng.bit_generator.state = state
            for _ in range(used):
                rng.integers(0, 2, size=payload_len, dtype=np.int8)
                rng.normal(0.0, noise_sigma, size=sym_len)
        for f in range(used):
            stats.update(int(bit_err[f]), float(work[f]), bool(bit_err[f] > 0), payload_len)
    row = stats.row()
    row.update({"scheme": args.scheme, "code": args.scheme, "N_or_E": coded_len, "K_payload": payload_len,
                "K_crc": args.K_crc, "rate": payload_len / coded_len, "params": params_label, "EbN0_dB": EbN0_dB})
    return row


def payload_errors_from_words(best: np.ndarray, ref: np.ndarray, K_payload: int) -> np.ndarray:
    """Per-frame payload bit errors (run_ber_sweep.py:77-82 on bit-packed words): popcount of
    best ^ ref over the first K_payload bits (bit j in word j >> 6, bit j & 63)."""
    best = np.asarray(best, np.uint64)
    ref = np.asarray(ref, np.uint64)
    W = best.shape[1]
    mask = np.zeros(W, np.uint64)
    for w in range(W):
        nb = min(max(K_payload - 64 * w, 0), 64)
        mask[w] = np.uint64((1 << nb) - 1) if nb < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
    return np.bitwise_count((best ^ ref) & mask).sum(axis=1).astype(np.int64)


class PhiloxFrames:
    """Frames [frame0, frame0 + n) of the on-device Philox stream of one SNR point, decoded on
    this rank's GPU: returns per-frame payload bit errors and work (flips tried for dl_scl)."""

    def __init__(self, args, info_set, N: int, device: int):
        a = self.args = args
        self.N, self.payload_len = N, a.K_payload
        crc = a.crc_poly if a.K_crc else None
        if a.scheme == "nr_polar_scl":
            crc = a.crc_poly  # scl_nr.py: always CRC-protected
        self.crc = crc
        E = a.E if a.scheme == "nr_polar_scl" else 0
        self.dec = _native.Decoder(N, info_set, a.M, crc, device)
        if E:
            self.dec.set_rate_match(E)
        self.n_in = E or N
        self.beta = np.load(a.beta) if (a.scheme == "dl_scl" and a.beta) else None
        self.mem = None
        self.cap = 0

    def _ensure(self, n: int) -> None:
        if n <= self.cap:
            return
        if self.mem is not None:
            self.mem.__exit__(None, None, None)
        W = self.dec.W
        self.mem = _native.DeviceArena(self.dec)
        self.d_llr = self.mem.alloc(n * self.n_in * 8)
        self.d_msg = self.mem.alloc(n * W * 8)
        self.d_best = self.mem.alloc(n * W * 8)
        self.d_flags = self.mem.alloc(n)
        self.d_att = self.mem.alloc(n * 4)
        self.cap = n

    def frames(self, seed: int, EbN0_dB: float, frame0: int, n: int):
        a, dec = self.args, self.dec
        if n <= 0:
            return np.zeros(0, np.int64), np.zeros(0)
        self._ensure(n)
        W = dec.W
        k_tx = self.payload_len  # payload bits; the CRC (if any) follows them
        dec.channel_device(seed, philox_stream_id(EbN0_dB), EbN0_dB, self.payload_len / a.E, k_tx, frame0, n,
                           self.d_llr, self.d_msg)
        work = np.zeros(n)
        if a.scheme == "dl_scl" and self.crc is not None:
            dec.dlscl_device(self.d_llr, n, a.retries, beta=self.beta, d_best=self.d_best, d_flags=self.d_flags,
                             d_attempts=self.d_att)
            dec.sync()
            work = (self.mem.download(self.d_att, n * 4, np.int32) - 1).astype(np.float64)
        else:
            dec.decode_device(self.d_llr, n, d_best=self.d_best, d_flags=self.d_flags)
            dec.sync()
        best = self.mem.download(self.d_best, n * W * 8, np.uint64).reshape(n, W)
        msg = self.mem.download(self.d_msg, n * W * 8, np.uint64).reshape(n, W)
        return payload_errors_from_words(best, msg, self.payload_len), work

    def close(self) -> None:
        if self.mem is not None:
            self.mem.__exit__(None, None, None)
            self.mem = None
        self.dec.close()


def run_scheme_philox(source, EbN0_dB, args, coded_len, payload_len, params_label, ctx=None) -> Dict:
    """One SNR point with frames from the counter-based device stream, sharded over ranks, with
    the reference's stop rule (run_ber_sweep.py:127) applied at the exact global frame."""
    ctx = ctx or dist.Context()
    stats = SimulationStats()
    frame = 0  # next global frame index of this SNR point
    while stats.bit_errors < args.err_cap and stats.bits_total < args.bits_cap:
        left = max(1, math.ceil((args.bits_cap - stats.bits_total) / payload_len))
        # philox: 2^16 frames per GPU per round by default -- a round's fixed cost (launches, the
        # all-gather, the host copy of per-frame errors) outweighs decoding a few thousand frames,
        # and the stop frame is exact whatever the round size (rows identical at any batch)
        total = int(min((args.batch or (1 << 16)) * ctx.world, left))
        s, e = dist.shard(total, ctx.rank, ctx.world)
        bit_err, work = source.frames(args.seed, EbN0_dB, frame + s, e - s)
        part = np.array([e - s, bit_err.sum(), np.count_nonzero(bit_err), work.sum()], np.float64)
        parts = dist.allgather(part, ctx)  # [world, 4], rank order
        err_round = int(parts[:, 1].sum())
        if stats.bit_errors + err_round < args.err_cap and stats.bits_total + total * payload_len < args.bits_cap:
            tot = parts.sum(axis=0)
            n_used, err_used, ferr_used, work_used = int(tot[0]), int(tot[1]), int(tot[2]), float(tot[3])
        else:  # the stop frame lies in this round: first global frame meeting the rule
            before = stats.bit_errors + int(parts[: ctx.rank, 1].sum())
            cum_err = before + np.cumsum(bit_err)
            cum_bits = stats.bits_total + payload_len * (s + np.arange(1, e - s + 1))
            hit = np.flatnonzero((cum_err >= args.err_cap) | (cum_bits >= args.bits_cap))
            cand = s + int(hit[0]) if hit.size else total
            stop = int(dist.allreduce_min(cand, ctx))  # round-local index of the last frame drawn
            k = int(np.clip(stop + 1 - s, 0, e - s))
            mine = np.array([k, bit_err[:k].sum(), np.count_nonzero(bit_err[:k]), work[:k].sum()], np.float64)
            tot = dist.allreduce_sum(mine, ctx)
            n_used, err_used, ferr_used, work_used = int(tot[0]), int(tot[1]), int(tot[2]), float(tot[3])
        stats.bits_total += n_used * payload_len
        stats.bit_errors += err_used
        stats.frame_errors += ferr_used
        stats.work_sum += work_used
        stats.frames += n_used
        frame += total
    row = stats.row()
    row.update({"scheme": args.scheme, "code": args.scheme, "N_or_E": coded_len, "K_payload": payload_len,
                "K_crc": args.K_crc, "rate": payload_len / coded_len, "params": params_label, "EbN0_dB": EbN0_dB})
    return row


def parse_args(argv: Optional[Iterable[str]] = None) -> argparse.Namespace:
    parser = argparse.ArgumentParser(description="BER/FER sweep across schemes")
    parser.add_argument("--scheme", required=True, choices=["polar_scl", "dl_scl", "nr_polar_scl", "nr_ldpc"],
                        help="Coding scheme")
    parser.add_argument("--K_payload", type=int, required=True, help="Payload bits per frame")
    parser.add_argument("--K_crc", type=int, required=True, help="CRC bits per frame")
    parser.add_argument("--E", type=int, required=True, help="Coded bits transmitted")
    parser.add_argument("--N", type=int, help="Polar length before rate match (defaults to E)")
    parser.add_argument("--crc_poly", type=str, default=global_config.DEFAULTS.crc_poly)
    parser.add_argument("--M", type=int, default=4, help="List size for polar decoders")
    parser.add_argument("--retries", type=int, default=8, help="Retries for DL-SCL")
    parser.add_argument("--beta", type=str, help="Path to beta matrix (DL-SCL)")
    parser.add_argument("--ilv_mode", type=str, default="default")
    parser.add_argument("--bg", type=int, default=2, help="LDPC base graph")
    parser.add_argument("--Z", type=int, default=2, help="LDPC lifting size")
    parser.add_argument("--max_iter", type=int, default=20)
    parser.add_argument("--alpha", type=float, default=0.8)
    parser.add_argument("--EbN0_lo", type=float, required=True)
    parser.add_argument("--EbN0_hi", type=float, required=True)
    parser.add_argument("--EbN0_step", type=float, default=0.5)
    parser.add_argument("--bits_cap", type=float, default=1e7)
    parser.add_argument("--err_cap", type=int, default=1000)
    parser.add_argument("--seed", type=int, default=0)
    parser.add_argument("--out", type=str, required=True, help="CSV output path")
    parser.add_argument("--plot", type=str, help="Optional plot path")
    # engine options (not in the reference)
    parser.add_argument("--batch", type=int, default=None,
                        help="frames per GPU batch (default 4096 with --rng replay, 2^16 with philox)")
    parser.add_argument("--device", type=int, default=0, help="GPU (single process; torchrun ranks use LOCAL_RANK)")
    parser.add_argument("--rng", choices=["replay", "philox"], default="replay",
                        help="replay: the reference's NumPy stream, exact rows, one process; philox: frames "
                             "generated on the GPU by global index, sharded over torchrun ranks")
    args = parser.parse_args(list(argv) if argv is not None else None)
    if args.scheme == "dl_scl" and not args.beta:
        raise ValueError("--beta is required for dl_scl scheme")
    return args


def run(args: argparse.Namespace) -> List[Dict[str, float]]:
    seed_all(args.seed)
    rng = np.random.default_rng(args.seed)
    N = args.N if args.N is not None else args.E
    K_total = args.K_payload + args.K_crc
    if args.scheme == "nr_ldpc":
        raise NotImplementedError("nr_ldpc (the reference's demo LDPC chain) is outside this engine's scope")
    info_set = construct_info_set(N, K_total)
    if args.scheme == "polar_scl":
        params_label = f"M={args.M}"
    elif args.scheme == "dl_scl":
        params_label = f"M={args.M},retries={args.retries}"
    else:
        params_label = f"M={args.M},ilv={args.ilv_mode}"
    snrs = np.arange(args.EbN0_lo, args.EbN0_hi + 1e-12, args.EbN0_step)
    rows: List[Dict[str, float]] = []
    if args.rng == "philox":
        ctx = dist.init()
        source = PhiloxFrames(args, info_set, N, ctx.device if ctx.world > 1 else args.device)
        try:
            for EbN0_dB in snrs:
                rows.append(run_scheme_philox(source, float(EbN0_dB), args, args.E, args.K_payload, params_label, ctx))
        finally:
            source.close()
        return rows
    if dist.init().world > 1:
        raise ValueError("--rng replay draws every frame from one NumPy stream (one process); "
                         "use --rng philox to shard frames over ranks")
    scheme = _Scheme(args, info_set, N)
    for EbN0_dB in snrs:
        rows.append(run_scheme(rng, float(EbN0_dB), args, info_set, scheme, args.E, args.K_payload, params_label))
    return rows


def write_csv(rows: List[Dict[str, float]], path: Path) -> None:
    """run_ber_sweep.py:296-317."""
    if not rows:
        return
    header = ["scheme", "code", "N_or_E", "K_payload", "K_crc", "rate", "params", "EbN0_dB", "bits_total",
              "bit_errors", "ber", "fer", "avg_work"]
    with path.open("w") as f:
        f.write(",".join(header) + "\n")
        for row in rows:
            f.write(",".join(str(row[col]) for col in header) + "\n")


def plot_rows(rows: List[Dict[str, float]], path: Path) -> None:
    if not rows:
        return
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        print("matplotlib not available; skipping plot")
        return
    rows_sorted = sorted(rows, key=lambda r: r["EbN0_dB"])
    snrs = [r["EbN0_dB"] for r in rows_sorted]
    plt.figure(figsize=(6, 4))
    plt.semilogy(snrs, [r["ber"] for r in rows_sorted], "o-", label="BER")
    plt.semilogy(snrs, [r["fer"] for r in rows_sorted], "s-", label="FER")
    plt.xlabel("Eb/N0 (dB)")
    plt.ylabel("Error Rate")
    plt.grid(True, which="both", ls="--", alpha=0.4)
    plt.legend()
    plt.tight_layout()
    path.parent.mkdir(parents=True, exist_ok=True)
    plt.savefig(path, dpi=200)
    plt.close()


def main(argv: Optional[Iterable[str]] = None) -> None:
    args = parse_args(argv)
    rows = run(args)
    if dist.init().is_root:
        out_path = Path(args.out)
        out_path.parent.mkdir(parents=True, exist_ok=True)
        write_csv(rows, out_path)
        if args.plot:
            plot_rows(rows, Path(args.plot))
    dist.finalize()


if __name__ == "__main__":
    main()
