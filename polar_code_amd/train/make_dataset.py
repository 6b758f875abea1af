"""Flip-label dataset for beta training (mirror of dl_scl_polar/train/make_dataset.py:24-141).

    python -m polar_code_amd.train.make_dataset --M 8 --snr_db 5.0 --frames 1000000 --out data/ds

Same CLI, same shard (``{out}_part0.npz``: ``abs_l0`` float32[S, K], ``flip_idx`` int32[S],
``meta`` JSON) and, in the default replay mode, the same samples as the reference:

* all-zero payload, CRC attached, encoded, BPSK; noise from ``default_rng(seed)`` drawn in the
  reference's order (one N-vector per frame), ``llr = 2 (x + n) / sigma^2``;
* baseline SCL on the GPU for a whole batch; frames whose best candidate passes the CRC are
  skipped (:63-64);
* for the failing frames: ``|L0|`` = the best path's decision LLRs cast to float32 (:66),
  their ``np.argsort`` order (:71), and up to min(8, K) flips tried in that order, each
  forcing the *baseline* best bits' prefix (:74-82, not chained like decode_with_retries).
  All failing frames of a batch are re-decoded together, one GPU batch per flip rank; a frame
  is labelled by the first flip whose result passes the CRC and equals the sent message
  (:86-88); frames without such a flip count as failures.

``--rng philox`` generates the frames on the GPU (counter-based, independent of batching)
and maps them to the all-zero codeword by the channel's symmetry (LLR sign flip where the
sent bit is 1: same noise law), for datasets far larger than the NumPy stream makes sense for.
"""
from __future__ import annotations

import argparse
import json
from pathlib import Path
from typing import List, Optional

import numpy as np

from .. import _native, config
from ..polar.crc import attach_crc
from ..polar.polar import construct_info_set, encode
from ..utils.seeding import seed_all


def decode_batch(llr: np.ndarray, info_set, M: int, crc, forced: Optional[np.ndarray] = None):
    """(best bits [B, K] int8, CRC pass [B] bool) of decode_scl for a batch (GPU)."""
    dec = _native.get_decoder(llr.shape[1], info_set, M, crc)
    out = dec.decode(llr, forced, want_metrics=False, want_cands=False, want_info_llrs=False)
    return out["best_bits"], out["crc_pass"]


def best_path_llrs(llr: np.ndarray, info_set, M: int, crc, bits: np.ndarray) -> np.ndarray:
    """best_path_info_llrs [B, K] of the paths with information bits `bits` (GPU replay)."""
    return _native.get_decoder(llr.shape[1], info_set, M, crc).path_llrs(llr, bits)


def _force_prefix_flip(bits: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """Rows of flip.py:30-34: bits[:i] forced, bit i flipped, the rest free (-1)."""
    B, K = bits.shape
    col = np.arange(K)[None, :]
    i = idx[:, None]
    forced = np.where(col < i, bits, np.int8(-1)).astype(np.int8)
    forced[np.arange(B), idx] = 1 - bits[np.arange(B), idx]
    return forced


def label_batch(llr: np.ndarray, info_set, M: int, crc: str, sent: np.ndarray):
    """Samples of one batch, in frame order: (abs_l0 float32 [S, K], labels int32 [S], failures)."""
    bits, ok = decode_batch(llr, info_set, M, crc)
    fail = np.flatnonzero(~ok)
    K = bits.shape[1]
    if fail.size == 0:
        return np.zeros((0, K), np.float32), np.zeros(0, np.int32), 0
    base = bits[fail]
    l0 = best_path_llrs(llr[fail], info_set, M, crc, base)
    abs_l0 = np.abs(np.asarray(l0, dtype=np.float32))
    order = np.stack([np.argsort(row) for row in abs_l0])  # per frame, as make_dataset.py:71
    label = np.full(fail.size, -1, np.int32)
    for t in range(min(8, K)):
        todo = np.flatnonzero(label < 0)
        if todo.size == 0:
            break
        idx = order[todo, t]
        cand, cpass = decode_batch(llr[fail[todo]], info_set, M, crc, _force_prefix_flip(base[todo], idx))
        hit = cpass & np.all(cand == sent[None, :], axis=1)
        label[todo[hit]] = idx[hit]
    keep = label >= 0
    return abs_l0[keep], label[keep], int(np.count_nonzero(~keep))


def _philox_frames(seed: int, snr_db: float, frame0: int, n: int, info_set, M: int, crc: str, kp: int):
    """n frames from the device TX chain, mapped to the all-zero codeword."""
    cfg = config.get_config()
    dec = _native.get_decoder(cfg.N, info_set, M, crc)
    W = dec.W
    with _native.DeviceArena(dec) as mem:
        d_llr = mem.alloc(n * cfg.N * 8)
        d_msg = mem.alloc(n * W * 8)
        dec.channel_device(seed, 0x7FFF0000 + int(round(snr_db * 10)), snr_db, cfg.K / cfg.N, kp, frame0, n, d_llr,
                           d_msg)
        llr = mem.download(d_llr, n * cfg.N * 8, np.float64).reshape(n, cfg.N)
        words = mem.download(d_msg, n * W * 8, np.uint64).reshape(n, W)
    msg = ((words[:, :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).reshape(n, -1)[:, :cfg.K]
    x = encode(msg.astype(np.int8))
    return llr * (1.0 - 2.0 * x)


def generate_samples(args: argparse.Namespace) -> Path:
    cfg = config.get_config()
    seed_all(args.seed)
    info_set = construct_info_set(cfg.N, cfg.K)
    payload_bits = cfg.K - cfg.crc_bits
    sent = attach_crc(np.zeros(payload_bits, dtype=np.int8), cfg.crc_poly)
    symbols = 1.0 - 2.0 * encode(sent)
    rate = cfg.K / cfg.N
    noise_var = 1.0 / (2.0 * rate * 10 ** (args.snr_db / 10.0))
    sigma = np.sqrt(noise_var)
    rng = np.random.default_rng(args.seed)

    xs: List[np.ndarray] = []
    ys: List[np.ndarray] = []
    failures = 0
    for b0 in range(0, args.frames, args.batch):
        n = min(args.batch, args.frames - b0)
        if args.rng == "replay":
            noise = rng.normal(0.0, sigma, size=(n, cfg.N))  # = n successive size-N draws
            llr = 2.0 * (symbols[None, :] + noise) / noise_var
        else:
            llr = _philox_frames(args.seed, args.snr_db, b0, n, info_set, args.M, cfg.crc_poly, payload_bits)
        a, lab, nf = label_batch(llr, info_set, args.M, cfg.crc_poly, sent)
        xs.append(a)
        ys.append(lab)
        failures += nf
    abs_array = np.concatenate(xs).astype(np.float32)
    label_array = np.concatenate(ys).astype(np.int32)
    if label_array.size == 0:
        raise RuntimeError("No samples collected; consider increasing frames or SNR")
    meta = {"M": args.M, "EbN0_dB": args.snr_db, "seed": args.seed, "frames": args.frames,
            "crc_poly": cfg.crc_poly, "crc_bits": cfg.crc_bits, "samples": int(label_array.size),
            "failures": int(failures)}
    out = Path(args.out)
    out_dir = out.parent if out.parent != Path("") else Path(".")
    out_dir.mkdir(parents=True, exist_ok=True)
    shard = out_dir / f"{out.name}_part0.npz"
    np.savez_compressed(shard, abs_l0=abs_array, flip_idx=label_array, meta=json.dumps(meta))
    print(f"Saved {label_array.size} samples to {shard}")
    return shard


def build_argparser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Generate DL-SCL flip dataset")
    p.add_argument("--M", type=int, required=True, help="SCL list size")
    p.add_argument("--snr_db", type=float, default=5.0, help="AWGN Eb/N0 in dB")
    p.add_argument("--frames", type=int, default=100000, help="Number of frames to simulate")
    p.add_argument("--seed", type=int, default=0, help="RNG seed")
    p.add_argument("--out", type=str, required=True, help="Output prefix for dataset shards")
    # engine options (not in the reference)
    p.add_argument("--rng", choices=["replay", "philox"], default="replay",
                   help="replay: the reference's NumPy stream (identical samples); philox: GPU-generated frames")
    p.add_argument("--batch", type=int, default=1 << 16, help="frames per GPU batch")
    return p


def main(argv: list[str] | None = None) -> None:
    generate_samples(build_argparser().parse_args(argv))


if __name__ == "__main__":
    main()
