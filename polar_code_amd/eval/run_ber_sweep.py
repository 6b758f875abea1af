"""BER/FER sweeps across schemes (mirror of dl_scl_polar/eval/run_ber_sweep.py: same flags,
rows and CSV).  Schemes polar_scl, dl_scl and nr_polar_scl decode on the GPU; nr_ldpc (the
reference's 3x6 demo base graph) is out of scope.

The reference draws every frame from ONE NumPy stream shared by all SNR points
(run_ber_sweep.py:230) and stops each point on a data-dependent rule
(`while bit_errors < err_cap and bits_total < bits_cap`, :127).  Here frames are generated in
batches from that same stream and decoded in one GPU call; the exact stop frame is found with
a prefix sum, and if a batch overshoots, the stream is rewound to the batch start and advanced
by exactly the frames the reference would have drawn -- so the rows (and the stream handed to
the next SNR point) are identical to the reference's.
"""
from __future__ import annotations

import argparse
import math
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, Iterable, List, Optional

import numpy as np

from .. import _native
from .. import config as global_config
from ..dlscl.flip import decode_with_retries_batch
from ..nr.polar.interleaver import subblock_interleave
from ..polar import polar as polar_core
from ..polar.crc import attach_crc
from ..polar.polar import construct_info_set
from ..utils.seeding import seed_all


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
        B = int(min(args.batch, left))
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
    parser.add_argument("--batch", type=int, default=4096, help="frames per GPU batch")
    parser.add_argument("--device", type=int, default=0)
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
    scheme = _Scheme(args, info_set, N)
    rows: List[Dict[str, float]] = []
    for EbN0_dB in np.arange(args.EbN0_lo, args.EbN0_hi + 1e-12, args.EbN0_step):
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
    out_path = Path(args.out)
    out_path.parent.mkdir(parents=True, exist_ok=True)
    write_csv(rows, out_path)
    if args.plot:
        plot_rows(rows, Path(args.plot))


if __name__ == "__main__":
    main()
