"""Reference-side binding of libpolar_mi355x.so -- the file a maintainer adds to the reference
as dl_scl_polar/polar/scl_mi355x.py.

Self-contained: ctypes and NumPy only, no import of polar_code_amd.  It replaces
  dl_scl_polar.polar.scl.decode_scl           (scl.py:108-209)
  dl_scl_polar.polar.polar.sc_decode           (polar.py:130-168)
and adds the batch API the host keeps (SCLDecoder: one call decodes llr[B, N], the
dl_scl_polar.polar.scl SCLDecoder contract of polar_code_amd/polar/scl.py) and a batch form of
dl_scl_polar.dlscl.flip.decode_with_retries (flip.py:65-141) whose retry loop runs on the GPU.  Return values and exception types follow the reference.

The library is found through $PSCL_LIB, else next to this repository's package.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_LIB_PATH = os.environ.get("PSCL_LIB") or str(Path(__file__).resolve().parent.parent / "polar_code_amd" /
                                              "libpolar_mi355x.so")
_vp, _i64, _i32 = C.c_void_p, C.c_int64, C.c_int32
_lib = C.CDLL(_LIB_PATH)
_lib.pscl_last_error.restype = C.c_char_p
_lib.pscl_create.argtypes = [C.POINTER(_vp), C.c_int, C.c_int, C.POINTER(_i32), C.c_int, C.c_int, C.c_uint64]
_lib.pscl_decode.argtypes = [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
_lib.pscl_sc_decode.argtypes = [_vp, _vp, _i64, _vp]
_lib.pscl_set_beta.argtypes = [_vp, _vp]
_lib.pscl_dlscl_device.argtypes = [_vp, _vp, _i64, C.c_int, _vp, _vp, _vp, _vp, C.c_int, _vp, C.c_int, _vp, _vp]
_lib.pscl_device_alloc.argtypes = [_vp, C.POINTER(_vp), _i64]
_lib.pscl_device_free.argtypes = [_vp, _vp]
_lib.pscl_memcpy_htod.argtypes = [_vp, _vp, _vp, _i64]
_lib.pscl_memcpy_dtoh.argtypes = [_vp, _vp, _vp, _i64]
_lib.pscl_sync.argtypes = [_vp]

_EINVAL, _EPRUNED, _EUNSUP = -1, -4, -5
_FLAG_CRC_PASS, _FLAG_IDX_MASK = 0x80, 0x3F
_handles: dict = {}


def _check(rc: int) -> None:
    if rc == 0:
        return
    msg = _lib.pscl_last_error().decode()
    if rc == _EINVAL:
        raise ValueError(msg)
    if rc == _EPRUNED:
        raise RuntimeError("All paths pruned during decoding")
    if rc == _EUNSUP:
        raise NotImplementedError(msg)
    raise RuntimeError(msg)


def _crc_value(crc) -> int:
    if crc is None:
        return 0
    return int(crc, 16) if isinstance(crc, str) else int(crc)


def _handle(N: int, info_set: np.ndarray, M: int, crc, device: int = 0):
    info = np.ascontiguousarray(np.asarray(info_set).ravel(), dtype=np.int32)
    key = (N, info.tobytes(), M, _crc_value(crc), int(device))
    if key not in _handles:
        h = _vp()
        _check(_lib.pscl_create(C.byref(h), int(device), N, info.ctypes.data_as(C.POINTER(_i32)), info.size, M,
                                _crc_value(crc)))
        _handles[key] = h
    return _handles[key]


def decode_scl(llr, info_set, M, crc=None, *, force_info_bits=None):
    """scl.py:108-209 on the GPU: candidates / metrics / info_llrs in list order, best path =
    first CRC-passing candidate, else the first (scl.py:190-201)."""
    if M <= 0:
        raise ValueError("List size M must be positive")
    llr = np.ascontiguousarray(np.asarray(llr, dtype=float).ravel())
    info_set = np.asarray(info_set)
    K = info_set.size
    forced = None
    if force_info_bits is not None:
        forced = np.ascontiguousarray(np.asarray(force_info_bits).ravel(), dtype=np.int8)
        if forced.size != K:
            raise ValueError("force_info_bits must have length equal to info_set")
    h = _handle(llr.size, info_set, M, crc)
    n = np.zeros(1, np.int32)
    best = np.zeros(1, np.int32)
    mets = np.zeros(M)
    cands = np.zeros((M, K), np.int8)
    illr = np.zeros((M, K))
    _check(_lib.pscl_decode(h, llr.ctypes.data, 1, None if forced is None else forced.ctypes.data, n.ctypes.data,
                            None, None, best.ctypes.data, mets.ctypes.data, cands.ctypes.data, illr.ctypes.data))
    k, b = int(n[0]), int(best[0])
    return {"candidates": [cands[i].copy() for i in range(k)], "metrics": [float(m) for m in mets[:k]],
            "best_path_bits": cands[b].copy(), "info_llrs": [illr[i].copy() for i in range(k)],
            "best_path_info_llrs": illr[b].copy()}


def sc_decode(llr, info_set):
    """polar.py:130-168 on the GPU: hard-decision successive cancellation, u[info_set]."""
    llr = np.ascontiguousarray(np.asarray(llr, dtype=float).ravel())
    info_set = np.asarray(info_set)
    h = _handle(llr.size, info_set, 1, None)
    bits = np.zeros(info_set.size, np.int8)
    _check(_lib.pscl_sc_decode(h, llr.ctypes.data, 1, bits.ctypes.data))
    return bits


class SCLDecoder:
    """Frame-batched SCL decoder bound to one GPU (scl.py:108-209 over a batch).

    SCLDecoder(N, info_set, L, crc_poly="0x1864CFB", device=0).decode(llr[B, N]) returns a dict
    with bits [B, K] int8 (each frame's best_path_bits), crc_pass [B] bool, best_idx [B] and
    n_paths [B]; with metrics / candidates / info_llrs=True also metrics [B, L] (list order),
    cands [B, L, K] and info_llrs [B, L, K].  forced: None or [B, K] int8 in {-1, 0, 1}
    (force_info_bits per frame: -1 free, 0/1 forced, scl.py:131-133).  One pscl_decode call per batch.
    """

    def __init__(self, N: int, info_set, L: int, crc_poly="0x1864CFB", device: int = 0):
        if L <= 0:
            raise ValueError("List size M must be positive")
        self.N, self.L, self.device = int(N), int(L), int(device)
        self.info_set = np.ascontiguousarray(np.asarray(info_set).ravel(), dtype=np.int32)
        self.K = self.info_set.size
        self.crc_poly = crc_poly
        self._h = _handle(self.N, self.info_set, self.L, crc_poly, self.device)

    def decode(self, llr, forced=None, *, metrics: bool = False, candidates: bool = False,
               info_llrs: bool = False) -> dict:
        llr = np.ascontiguousarray(np.asarray(llr, dtype=float))
        if llr.ndim == 1:
            llr = llr[None, :]
        if llr.ndim != 2 or llr.shape[1] != self.N:
            raise ValueError(f"llr must be [B, {self.N}]")
        B, K, L = llr.shape[0], self.K, self.L
        if forced is not None:
            forced = np.ascontiguousarray(np.asarray(forced), dtype=np.int8)
            if forced.shape != (B, K):
                raise ValueError("force_info_bits must have length equal to info_set")
        out = {"n_paths": np.zeros(B, np.int32), "bits": np.zeros((B, K), np.int8),
               "crc_pass": np.zeros(B, np.uint8), "best_idx": np.zeros(B, np.int32)}
        if metrics:
            out["metrics"] = np.full((B, L), np.nan)
        if candidates:
            out["cands"] = np.zeros((B, L, K), np.int8)
        if info_llrs:
            out["info_llrs"] = np.full((B, L, K), np.nan)

        def p(k):
            a = out.get(k)
            return None if a is None else a.ctypes.data

        _check(_lib.pscl_decode(self._h, llr.ctypes.data, B, None if forced is None else forced.ctypes.data,
                                p("n_paths"), p("bits"), p("crc_pass"), p("best_idx"), p("metrics"), p("cands"),
                                p("info_llrs")))
        out["crc_pass"] = out["crc_pass"].astype(bool)
        return out


class _Device:
    """Device buffers of one call, freed on exit."""

    def __init__(self, h):
        self.h, self.ptrs = h, []

    def alloc(self, nbytes: int) -> int:
        p = _vp()
        _check(_lib.pscl_device_alloc(self.h, C.byref(p), max(int(nbytes), 1)))
        self.ptrs.append(p.value)
        return p.value

    def put(self, arr: np.ndarray) -> int:
        arr = np.ascontiguousarray(arr)
        p = self.alloc(arr.nbytes)
        _check(_lib.pscl_memcpy_htod(self.h, p, arr.ctypes.data, arr.nbytes))
        return p

    def get(self, p: int, shape, dtype) -> np.ndarray:
        out = np.zeros(shape, dtype)
        _check(_lib.pscl_memcpy_dtoh(self.h, out.ctypes.data, p, out.nbytes))
        return out

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        for p in self.ptrs:
            _lib.pscl_device_free(self.h, p)


def decode_with_retries_batch(llr, info_set, M, retries, *, crc=None, beta=None):
    """decode_with_retries (flip.py:65-141) for a batch llr[B, N], the retry loop on the GPU.
    Returns best_path_bits [B, K] (final attempt), success [B], attempts [B] and
    tried_indices (list of B lists)."""
    llr = np.ascontiguousarray(np.asarray(llr, dtype=float))
    if llr.ndim == 1:
        llr = llr[None, :]
    B, N = llr.shape
    info_set = np.asarray(info_set)
    K = info_set.size
    W = (K + 63) // 64 if K else 1
    R = max(int(retries), 0)
    h = _handle(N, info_set, M, crc)
    b = None if beta is None else np.ascontiguousarray(beta, dtype=np.float64)
    _check(_lib.pscl_set_beta(h, None if b is None else b.ctypes.data))
    with _Device(h) as dev:
        d_llr = dev.put(llr)
        d_best, d_flags, d_att = dev.alloc(B * W * 8), dev.alloc(B), dev.alloc(B * 4)
        d_tried = dev.alloc(B * max(R, 1) * 4)
        _check(_lib.pscl_dlscl_device(h, d_llr, B, R, d_best, d_flags, d_att, d_tried if R else None, R, None, 0,
                                      None, None))
        _check(_lib.pscl_sync(h))
        words = dev.get(d_best, (B, W), np.uint64)
        flags = dev.get(d_flags, B, np.uint8)
        att = dev.get(d_att, B, np.int32)
        tried = dev.get(d_tried, (B, max(R, 1)), np.int32)[:, :R]
    sh = np.arange(64, dtype=np.uint64)
    bits = ((words[:, :, None] >> sh) & np.uint64(1)).reshape(B, -1)[:, :K].astype(np.int8)
    success = (flags & _FLAG_CRC_PASS) != 0 if crc is not None else np.ones(B, bool)
    return {"best_path_bits": bits, "success": success, "attempts": att,
            "tried_indices": [[int(t) for t in row if t >= 0] for row in tried]}


__all__ = ["decode_scl", "sc_decode", "SCLDecoder", "decode_with_retries_batch"]
