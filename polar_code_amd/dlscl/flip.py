"""DL-SCL bit-flip retries (mirror of dl_scl_polar/dlscl/flip.py:13-141).

Every decode runs on the GPU.  Two batch forms:
  decode_with_retries_device  the whole retry loop on the device (pscl_dlscl_device):
                              flip choice q = |L0| @ beta summed in index order, argmin over
                              untried indices (ties -> lower index), compaction per round.
  decode_with_retries_batch   GPU decodes, flip ranking on the host with exactly the
                              reference's numpy calls (argsort, BLAS order) per frame.
The two agree except where two q values of a frame tie within BLAS rounding (numpy's own
argsort/BLAS order is machine-dependent there); tests hold both to the golden traces.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from .. import _native
from ..polar.crc import check_crc
from ..polar.scl import decode_scl


def choose_flip_index(abs_l0: np.ndarray, beta: Optional[np.ndarray]) -> int:
    """Choose the flip index by the beta metric, else by |L0| (flip.py:13-27)."""
    if abs_l0.ndim != 1:
        raise ValueError("abs_l0 must be a 1D array")
    if abs_l0.size == 0:
        raise ValueError("abs_l0 cannot be empty")
    if beta is not None:
        if beta.ndim != 2 or beta.shape[0] != beta.shape[1] or beta.shape[0] != abs_l0.size:
            raise ValueError("beta must be a square matrix matching abs_l0 length")
        q = abs_l0 @ beta
        return int(np.argmin(q))
    return int(np.argmin(abs_l0))


def _force_vector(best_path_bits: np.ndarray, flip_index: int) -> np.ndarray:
    """Forced prefix + flipped bit, free suffix (flip.py:30-34)."""
    forced = np.full(best_path_bits.size, -1, dtype=np.int8)
    forced[:flip_index] = best_path_bits[:flip_index]
    forced[flip_index] = 1 - best_path_bits[flip_index]
    return forced


def _rank_indices(abs_l0: np.ndarray, beta: Optional[np.ndarray]) -> List[int]:
    # flip.py:104-108, identical numpy calls
    if beta is not None:
        return list(np.argsort(abs_l0 @ beta))
    return list(np.argsort(abs_l0))


def retry_with_flip(llr_root, info_set, M, best_path_bits, flip_index, crc=None, *, device: int = 0) -> dict:
    """Re-decode with info bit `flip_index` flipped and the prefix forced (flip.py:37-62)."""
    if best_path_bits.ndim != 1:
        raise ValueError("best_path_bits must be 1D")
    if flip_index < 0 or flip_index >= best_path_bits.size:
        raise IndexError("flip_index out of range")
    forced = _force_vector(best_path_bits, flip_index)
    result = decode_scl(llr_root, info_set, M, crc=crc, force_info_bits=forced, device=device)
    result["forced_info_bits"] = forced
    result["flip_index"] = flip_index
    return result


def decode_with_retries(llr_root, info_set, M, retries, *, crc=None, beta=None, device: int = 0) -> dict:
    """Baseline SCL then up to `retries` flip attempts (flip.py:65-141)."""
    attempts: List[dict] = []
    baseline = decode_scl(llr_root, info_set, M, crc=crc, device=device)
    attempts.append({**baseline, "attempt_type": "baseline"})
    best_output = baseline

    def _passes(output: dict) -> bool:
        if crc is None:
            return output.get("best_path_bits") is not None
        bits = output.get("best_path_bits")
        return bits is not None and check_crc(bits, crc)

    if _passes(baseline) or retries <= 0:
        return {**best_output, "attempts": attempts, "tried_indices": [], "success": _passes(best_output)}

    reference_bits = baseline.get("best_path_bits")
    reference_llrs = baseline.get("best_path_info_llrs")
    if reference_bits is None or reference_llrs is None:
        raise ValueError("Baseline decode did not produce candidate bits/LLRs")
    abs_l0 = np.abs(np.asarray(reference_llrs, dtype=float))
    tried: List[int] = []
    while len(tried) < retries and len(tried) < abs_l0.size:
        idx = next((i for i in _rank_indices(abs_l0, beta) if i not in tried), None)
        if idx is None:
            break
        tried.append(idx)
        retry_result = retry_with_flip(llr_root, info_set, M, reference_bits, flip_index=idx, crc=crc,
                                       device=device)
        attempts.append({**retry_result, "attempt_type": "flip"})
        best_output = retry_result
        if retry_result.get("best_path_bits") is not None:
            reference_bits = retry_result["best_path_bits"]
        if retry_result.get("best_path_info_llrs") is not None:
            reference_llrs = retry_result["best_path_info_llrs"]
        abs_l0 = np.abs(np.asarray(reference_llrs, dtype=float))
        if _passes(retry_result):
            break
    return {**best_output, "attempts": attempts, "tried_indices": tried, "success": _passes(best_output)}


def decode_with_retries_batch(llr: np.ndarray, info_set, M: int, retries: int, *, crc=None, beta=None,
                              device: int = 0, baseline: Optional[dict] = None) -> dict:
    """decode_with_retries for a batch [B, N], same per-frame results.

    Returns best_bits [B, K] int8 (the final attempt's best path, flip.py:126,137),
    success [B] bool, attempts [B] int32 (1 + retries used), tried [B, retries] int32 (-1 pad).
    `baseline` may carry an earlier decode of the same frames (keys best_bits, crc_pass).
    """
    llr = np.ascontiguousarray(llr, dtype=np.float64)
    B, N = llr.shape
    info_set = np.asarray(info_set)
    K = info_set.size
    dec = _native.get_decoder(N, info_set, M, crc, device)
    if baseline is None:
        baseline = dec.decode(llr, want_metrics=False, want_cands=False, want_info_llrs=False)
    bits = np.array(baseline["best_bits"], dtype=np.int8, copy=True)
    ok = np.asarray(baseline["crc_pass"], dtype=bool).copy() if crc is not None else np.ones(B, bool)
    attempts = np.ones(B, np.int32)
    tried = np.full((B, max(retries, 0)), -1, np.int32)
    active = np.flatnonzero(~ok) if retries > 0 else np.zeros(0, np.int64)
    if active.size:
        # |L0| of the baseline's best path for the failing frames (same decode, with history)
        again = dec.decode(llr[active], want_metrics=False, want_cands=False, want_info_llrs=True)
        ref_bits = again["best_bits"].copy()
        abs_l0 = np.abs(again["info_llrs"][np.arange(active.size), again["best_idx"]])
        ntried = np.zeros(active.size, np.int64)
        live = np.ones(active.size, bool)
        for _ in range(min(retries, K)):
            sel = np.flatnonzero(live)
            if sel.size == 0:
                break
            forced = np.full((sel.size, K), -1, np.int8)
            for r, a in enumerate(sel):
                seen = set(tried[active[a], : ntried[a]].tolist())
                idx = next((i for i in _rank_indices(abs_l0[a], beta) if i not in seen), None)
                tried[active[a], ntried[a]] = idx
                ntried[a] += 1
                forced[r] = _force_vector(ref_bits[a], int(idx))
            out = dec.decode(llr[active[sel]], forced, want_metrics=False, want_cands=False, want_info_llrs=True)
            fb = out["best_bits"]
            ref_bits[sel] = fb
            abs_l0[sel] = np.abs(out["info_llrs"][np.arange(sel.size), out["best_idx"]])
            bits[active[sel]] = fb
            attempts[active[sel]] += 1
            passed = out["crc_pass"] if crc is not None else np.ones(sel.size, bool)
            ok[active[sel]] = passed
            live[sel[passed]] = False
            live &= ntried < retries
    return {"best_bits": bits, "success": ok, "attempts": attempts, "tried": tried}


def bits_to_words(bits: np.ndarray) -> np.ndarray:
    """[B, K] 0/1 -> [B, W] uint64, bit j of word j // 64 = bits[:, j]."""
    bits = np.asarray(bits, dtype=np.uint64)
    B, K = bits.shape
    W = (K + 63) // 64 if K else 1
    out = np.zeros((B, W), np.uint64)
    for j in range(K):
        out[:, j >> 6] |= bits[:, j] << np.uint64(j & 63)
    return out


def words_to_bits(words: np.ndarray, K: int) -> np.ndarray:
    w = np.asarray(words, dtype=np.uint64)
    sh = np.arange(64, dtype=np.uint64)
    return ((w[:, :, None] >> sh) & np.uint64(1)).reshape(w.shape[0], -1)[:, :K].astype(np.int8)


def decode_with_retries_device(llr: np.ndarray, info_set, M: int, retries: int, *, crc=None, beta=None,
                               device: int = 0, msg: Optional[np.ndarray] = None,
                               tuning: Optional[dict] = None) -> dict:
    """decode_with_retries for a batch [B, N] with the retry loop on the GPU.

    Returns best_bits [B, K] (final attempt), success [B], attempts [B], tried [B, R]
    (R = max(retries, 0), -1 padded), base_bits / base_pass (the baseline SCL), and with
    `msg` [B, K] the in-kernel counters {"scl": [...], "dl": [...]} (PSCL_CNT_* order).
    `tuning`: schedule knobs for this call (Decoder.set_tuning; the handle's previous values,
    e.g. knobs a caller set on the shared decoder, are restored after).
    """
    llr = np.ascontiguousarray(llr, dtype=np.float64)
    B, N = llr.shape
    info_set = np.asarray(info_set)
    K = info_set.size
    dec = _native.get_decoder(N, info_set, M, crc, device)
    W = dec.W
    R = max(int(retries), 0)
    out = {}
    prev = dec.get_tuning() if tuning else {}
    if tuning:
        dec.set_tuning(**tuning)
    try:
        _retries_device(dec, llr, B, W, R, K, retries, crc, beta, msg, out)
    finally:
        if tuning:
            dec.set_tuning(**{k: prev.get(k, 0) for k in tuning})
    return out


def _retries_device(dec, llr, B, W, R, K, retries, crc, beta, msg, out) -> None:
    with _native.DeviceArena(dec) as mem:
        d_llr = mem.alloc(llr.nbytes)
        mem.upload(d_llr, llr)
        d_best = mem.alloc(B * W * 8)
        d_flags = mem.alloc(B)
        d_att = mem.alloc(B * 4)
        d_tried = mem.alloc(max(B * R * 4, 4))
        d_ref = d_cs = d_cd = 0
        if msg is not None:
            d_ref = mem.alloc(B * W * 8)
            mem.upload(d_ref, bits_to_words(msg))
            d_cs = mem.alloc(_native.PSCL_NCOUNT * 8)
            d_cd = mem.alloc(_native.PSCL_NCOUNT * 8)
            mem.memset(d_cs, 0, _native.PSCL_NCOUNT * 8)
            mem.memset(d_cd, 0, _native.PSCL_NCOUNT * 8)
        d_bbest = mem.alloc(B * W * 8)
        d_bflags = mem.alloc(B)
        dec.decode_device(d_llr, B, d_best=d_bbest, d_flags=d_bflags)
        dec.dlscl_device(d_llr, B, retries, beta=beta, d_best=d_best, d_flags=d_flags, d_attempts=d_att,
                         d_tried=d_tried if R else 0, tried_stride=R, d_ref=d_ref, k_payload=K - dec.crc_deg,
                         d_counters_scl=d_cs, d_counters_dl=d_cd)
        dec.sync()
        flags = mem.download(d_flags, B, np.uint8)
        bflags = mem.download(d_bflags, B, np.uint8)
        out["best_bits"] = words_to_bits(mem.download(d_best, B * W * 8, np.uint64).reshape(B, W), K)
        out["success"] = (flags & _native.PSCL_FLAG_CRC_PASS) != 0 if crc is not None else np.ones(B, bool)
        out["attempts"] = mem.download(d_att, B * 4, np.int32)
        out["tried"] = (mem.download(d_tried, B * R * 4, np.int32).reshape(B, R) if R
                        else np.zeros((B, 0), np.int32))
        out["base_bits"] = words_to_bits(mem.download(d_bbest, B * W * 8, np.uint64).reshape(B, W), K)
        out["base_pass"] = (bflags & _native.PSCL_FLAG_CRC_PASS) != 0 if crc is not None else np.ones(B, bool)
        if msg is not None:
            out["counters"] = {"scl": mem.download(d_cs, _native.PSCL_NCOUNT * 8, np.int64),
                               "dl": mem.download(d_cd, _native.PSCL_NCOUNT * 8, np.int64)}


__all__ = ["choose_flip_index", "retry_with_flip", "decode_with_retries", "decode_with_retries_batch",
           "decode_with_retries_device", "bits_to_words", "words_to_bits"]
