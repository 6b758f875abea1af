"""Successive-cancellation list decoding on the MI355X (mirror of dl_scl_polar/polar/scl.py).

`decode_scl` keeps the reference signature and return dict (scl.py:108-209) and runs one
frame through libpolar_mi355x.so.  `SCLDecoder` is the batch API the reference lacks: it
decodes [B, N] LLRs per call, on host arrays or on device-resident torch tensors.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from .. import _native


def _validate(llr, info_set, M, force_info_bits):
    if M <= 0:
        raise ValueError("List size M must be positive")
    info_set = np.asarray(info_set)
    if info_set.ndim != 1:
        raise ValueError("info_set must be a 1D array")
    if force_info_bits is not None:
        force_info_bits = np.asarray(force_info_bits)
        if force_info_bits.ndim != 1:
            raise ValueError("force_info_bits must be 1D when provided")
        if force_info_bits.size != info_set.size:
            raise ValueError("force_info_bits length must match info_set")
        force_info_bits = force_info_bits.astype(np.int8)
    llr = np.asarray(llr).astype(float).ravel()
    N = llr.size
    if N <= 0 or (N & (N - 1)):
        raise ValueError("Channel LLR length must be a power of two")
    return llr, info_set, force_info_bits


def decode_scl(
    llr: np.ndarray,
    info_set: np.ndarray,
    M: int,
    crc: Optional[str] = None,
    *,
    force_info_bits: Optional[np.ndarray] = None,
    device: int = 0,
) -> dict:
    """Decode one frame with SCL (list size M) and optional CRC selection (scl.py:108-209).

    Returns the reference's dict: candidates (list of int8[K], list order), metrics
    (list of float), best_path_bits (first CRC-passing candidate, else the first),
    info_llrs (decision LLR at each information phase, per candidate) and
    best_path_info_llrs.
    """
    llr, info_set, force = _validate(llr, info_set, M, force_info_bits)
    dec = _native.get_decoder(llr.size, info_set, int(M), crc, device)
    out = dec.decode(llr[None, :], None if force is None else force[None, :])
    n = int(out["n_paths"][0])
    candidates = [out["cands"][0, i].copy() for i in range(n)]
    metrics = [float(m) for m in out["metrics"][0, :n]]
    info_llrs = [out["info_llrs"][0, i].copy() for i in range(n)]
    b = int(out["best_idx"][0]) if n else None
    return {
        "candidates": candidates,
        "metrics": metrics,
        "best_path_bits": candidates[b] if b is not None else None,
        "info_llrs": info_llrs,
        "best_path_info_llrs": info_llrs[b] if b is not None else None,
    }


class SCLDecoder:
    """Frame-batched SCL decoder bound to one GPU.

    SCLDecoder(N, info_set, L, crc_poly="0x1864CFB", device=0).decode(llr[B, N]) returns a
    dict with bits [B, K] int8 (best_path_bits), crc_pass [B] bool, best_idx [B],
    n_paths [B], and, when requested, metrics [B, L], cands [B, L, K], info_llrs [B, L, K].
    """

    def __init__(self, N: int, info_set, L: int, crc_poly: Optional[str] = "0x1864CFB", device: int = 0):
        if L <= 0:
            raise ValueError("List size M must be positive")
        self.N, self.L, self.crc_poly, self.device = int(N), int(L), crc_poly, int(device)
        self.info_set = np.asarray(info_set).astype(np.int32)
        self.K = self.info_set.size
        self._dec = _native.Decoder(self.N, self.info_set, self.L, crc_poly, self.device)

    @property
    def native(self) -> _native.Decoder:
        return self._dec

    def decode(self, llr: np.ndarray, forced: Optional[np.ndarray] = None, *, metrics: bool = False,
               candidates: bool = False, info_llrs: bool = False) -> dict:
        out = self._dec.decode(llr, forced, want_metrics=metrics, want_cands=candidates,
                               want_info_llrs=info_llrs)
        out["bits"] = out.pop("best_bits")
        return {k: v for k, v in out.items() if v is not None}

    def decode_tensor(self, llr, forced_words=None, ref_words=None, k_payload: int = 0, counters=None):
        """Device path: llr is a contiguous float64 torch tensor [B, N] on this GPU.
        Returns (best_words [B, W] int64, flags [B] uint8) tensors; when ref_words is given,
        error statistics are added into `counters` (int64[8] tensor)."""
        import torch

        if llr.dtype != torch.float64 or not llr.is_contiguous() or llr.dim() != 2 or llr.shape[1] != self.N:
            raise ValueError("llr must be a contiguous float64 [B, N] tensor")
        B = llr.shape[0]
        W = self._dec.W
        best = torch.empty((B, W), dtype=torch.int64, device=llr.device)
        flags = torch.empty((B,), dtype=torch.uint8, device=llr.device)
        self._dec.set_stream(torch.cuda.current_stream(llr.device).cuda_stream)
        self._dec.decode_device(
            llr.data_ptr(), B,
            d_force=forced_words.data_ptr() if forced_words is not None else 0,
            d_best=best.data_ptr(), d_flags=flags.data_ptr(),
            d_ref=ref_words.data_ptr() if ref_words is not None else 0, k_payload=k_payload,
            d_counters=counters.data_ptr() if counters is not None else 0)
        return best, flags


__all__ = ["decode_scl", "SCLDecoder"]
