"""DL-SCL bit-flip retries (mirror of dl_scl_polar/dlscl/flip.py:13-141).

Every decode runs on the GPU.  The flip ranking (q = |L0| @ beta, argsort, first untried
index) stays on the host with exactly the reference's numpy calls -- per frame, on the
same shapes -- so the ranking (including its tie order and BLAS summation order) is the
reference's own.  `decode_with_retries_batch` is the throughput form used by the FER
sweep: one batched GPU decode per retry round over the frames that still fail.
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


__all__ = ["choose_flip_index", "retry_with_flip", "decode_with_retries", "decode_with_retries_batch"]
