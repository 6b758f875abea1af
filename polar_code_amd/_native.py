"""ctypes binding of libpolar_mi355x.so (include/polar_scl.h).

There is deliberately no fallback: if the HIP library is missing or no GPU is visible,
every decode raises.  Argument errors are mapped back to the reference's exception types
(ValueError / RuntimeError, dl_scl_polar/polar/scl.py:117-131,171-172).
"""
from __future__ import annotations

import ctypes as C
import functools
import importlib.util
import os
import sys
import threading
from pathlib import Path

import numpy as np

LIB_PATH = Path(os.environ.get("PSCL_LIB_PATH") or Path(__file__).resolve().parent / "libpolar_mi355x.so")

PSCL_OK = 0
PSCL_EINVAL = -1
PSCL_EDEVICE = -2
PSCL_ENOMEM = -3
PSCL_EPRUNED = -4
PSCL_EUNSUP = -5
PSCL_MAX_N = 1024
PSCL_REPLAY_MAX_N = 128  # pscl_path_llrs_device (decision-LLR replay); TX, decode and the DL-SCL loop take any N
PSCL_MAX_L = 32
PSCL_FLAG_CRC_PASS = 0x80
PSCL_FLAG_IDX_MASK = 0x3F
PSCL_NCOUNT = 8
CNT_FRAMES, CNT_FRAME_ERR, CNT_BIT_ERR, CNT_PAYLOAD_ERR, CNT_PAYLOAD_BIT, CNT_RETRIES = range(6)

# every symbol the header declares (tests/test_capi_symbols.py checks the .so exports them)
EXPORTS = (
    "pscl_last_error", "pscl_abi_version", "pscl_device_count", "pscl_create", "pscl_destroy",
    "pscl_set_stream", "pscl_get_stream", "pscl_sync", "pscl_decode", "pscl_sc_decode",
    "pscl_decode_device", "pscl_channel_device", "pscl_device_alloc", "pscl_device_free",
    "pscl_memcpy_htod", "pscl_memcpy_dtoh", "pscl_memset_device", "pscl_timing_enable",
    "pscl_timing_read", "pscl_launch_info", "pscl_set_rate_match", "pscl_set_beta", "pscl_dlscl_device",
    "pscl_path_llrs_device", "pscl_uncoded_device", "pscl_simulate", "pscl_set_screening", "pscl_build_hash",
    "pscl_screening_count", "pscl_softplus_tails_device", "pscl_set_pipelined", "pscl_join",
    "pscl_tail_abs_scan_device", "pscl_tail2_scan_device", "pscl_set_tuning", "pscl_timing_read_split", "pscl_decode_cpu",
    "pscl_host_stats", "pscl_path_stats",
    "pscl_simulate_device",
)

# pscl_set_tuning knobs (include/polar_scl.h)
TUNE = {"dl_screen": 1, "dl_chunks": 2, "dl_split": 3, "side_priority": 4, "post_grid": 5, "retry_wpg": 6, "dl_lane": 7, "dl_screen_min": 8, "dl_retry_lane": 9, "post_pairs": 10, "dl_streams": 11, "tx_fused": 12,
        "dl_fused_post": 13, "post_epw": 14, "lane_exact": 15, "dl_warm_apx": 16, "dl_tail": 17}

_vp, _i32, _i64, _u64, _dbl = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_double


class PolarNativeError(RuntimeError):
    """Device/runtime failure inside libpolar_mi355x.so."""


def _bind_hip_runtime() -> None:
    """Keep ONE HIP runtime per process.  PyTorch-ROCm bundles its own libamdhip64.so.7; if
    this library loaded /opt/rocm's copy first, torch would later load a second runtime and
    see no GPU.  Preloading torch's copy (same soname) makes both bind to it.  Set
    PSCL_HIP_RUNTIME=system to keep /opt/rocm's runtime (processes that never use torch)."""
    if os.environ.get("PSCL_HIP_RUNTIME", "") == "system" or "torch" in sys.modules:
        return
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    cand = Path(spec.origin).parent / "lib" / "libamdhip64.so"
    if cand.exists():
        C.CDLL(str(cand), mode=C.RTLD_GLOBAL)


def _check_fresh() -> None:
    """Refuse a library built from other sources than the ones in this tree (its embedded
    build hash, polar_code_amd/build.py).  Skipped where the sources are absent."""
    from . import build

    if not all((build.CSRC / s).exists() for s in build.HIP_DEPS):
        return
    want, got = build.source_hash(), build.library_hash(LIB_PATH)
    if got != want:
        raise PolarNativeError(
            f"{LIB_PATH} is stale (built from sources {got}, tree has {want}): "
            "run `python -m polar_code_amd.build`")


@functools.lru_cache(maxsize=1)
def lib() -> C.CDLL:
    _bind_hip_runtime()
    if not LIB_PATH.exists():
        raise PolarNativeError(
            f"{LIB_PATH} not built: run `python -m polar_code_amd.build` (hipcc, gfx950). "
            "There is no CPU fallback for the decoder.")
    if not os.environ.get("PSCL_LIB_PATH"):
        _check_fresh()
    L = C.CDLL(str(LIB_PATH))
    P = C.POINTER
    sig = {
        "pscl_last_error": (C.c_char_p, []),
        "pscl_abi_version": (C.c_int, []),
        "pscl_build_hash": (C.c_char_p, []),
        "pscl_screening_count": (C.c_int, [_vp, P(_i64)]),
        "pscl_set_pipelined": (C.c_int, [_vp, C.c_int]),
        "pscl_join": (C.c_int, [_vp]),
        "pscl_softplus_tails_device": (C.c_int, [_vp, _vp, _i64, _vp, _vp]),
        "pscl_tail_abs_scan_device": (C.c_int, [_vp, C.c_uint32, C.c_uint32, _vp]),
        "pscl_tail2_scan_device": (C.c_int, [_vp, C.c_uint32, C.c_uint32, _vp]),
        "pscl_set_tuning": (C.c_int, [_vp, C.c_int, _i64]),
        "pscl_simulate_device": (C.c_int, [_vp, _u64, C.c_uint32, _dbl, _dbl, C.c_int, _i64, _i64, C.c_int, C.c_int,
                                           _vp]),
        "pscl_decode_cpu": (C.c_int, [C.c_int, P(_i32), C.c_int, C.c_int, _u64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                      _vp, _vp, C.c_int]),
        "pscl_timing_read_split": (C.c_int, [_vp, P(_i64), P(_dbl), P(_i64), P(_dbl)]),
        "pscl_host_stats": (C.c_int, [_vp, P(_dbl), P(_dbl), P(_i64), C.c_int]),
        "pscl_path_stats": (C.c_int, [_vp, P(_i64), P(_i64), P(_i64), P(_i64), P(_i64)]),
        "pscl_device_count": (C.c_int, []),
        "pscl_create": (C.c_int, [P(_vp), C.c_int, C.c_int, P(_i32), C.c_int, C.c_int, _u64]),
        "pscl_destroy": (C.c_int, [_vp]),
        "pscl_set_stream": (C.c_int, [_vp, _vp]),
        "pscl_get_stream": (_vp, [_vp]),
        "pscl_sync": (C.c_int, [_vp]),
        "pscl_decode": (C.c_int, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
        "pscl_sc_decode": (C.c_int, [_vp, _vp, _i64, _vp]),
        "pscl_decode_device": (C.c_int, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int, _vp]),
        "pscl_channel_device": (C.c_int, [_vp, _u64, C.c_uint32, _dbl, _dbl, C.c_int, _i64, _i64, _vp, _vp]),
        "pscl_device_alloc": (C.c_int, [_vp, P(_vp), _i64]),
        "pscl_device_free": (C.c_int, [_vp, _vp]),
        "pscl_memcpy_htod": (C.c_int, [_vp, _vp, _vp, _i64]),
        "pscl_memcpy_dtoh": (C.c_int, [_vp, _vp, _vp, _i64]),
        "pscl_memset_device": (C.c_int, [_vp, _vp, C.c_int, _i64]),
        "pscl_timing_enable": (C.c_int, [_vp, C.c_int]),
        "pscl_set_screening": (C.c_int, [_vp, C.c_int]),
        "pscl_timing_read": (C.c_int, [_vp, P(_i64), P(_dbl)]),
        "pscl_launch_info": (C.c_int, [_vp, _i64, P(C.c_int), P(_i64), P(C.c_int)]),
        "pscl_set_rate_match": (C.c_int, [_vp, C.c_int]),
        "pscl_set_beta": (C.c_int, [_vp, _vp]),
        "pscl_path_llrs_device": (C.c_int, [_vp, _vp, _i64, _vp, _vp]),
        "pscl_uncoded_device": (C.c_int, [_vp, _u64, C.c_uint32, _dbl, C.c_int, _i64, _i64, _vp]),
        "pscl_simulate": (C.c_int, [_vp, _u64, C.c_uint32, _dbl, _dbl, C.c_int, _i64, _i64, C.c_int, C.c_int, _vp]),
        "pscl_dlscl_device": (C.c_int, [_vp, _vp, _i64, C.c_int, _vp, _vp, _vp, _vp, C.c_int, _vp, C.c_int, _vp,
                                        _vp]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("PSCL_LIB_PATH") and not hasattr(L, name):
            continue  # an older variant library under A/B timing (tools/ab_bench.sh)
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def build_hash() -> str:
    """The loaded library's embedded source hash ("" for variant libraries without one)."""
    fn = getattr(lib(), "pscl_build_hash", None)
    return fn().decode() if fn is not None else ""


def last_error() -> str:
    return lib().pscl_last_error().decode(errors="replace")


def check(rc: int) -> None:
    if rc == PSCL_OK:
        return
    msg = last_error()
    if rc == PSCL_EINVAL:
        raise ValueError(msg)
    if rc == PSCL_EPRUNED:
        raise RuntimeError("All paths pruned during decoding")
    if rc == PSCL_EUNSUP:
        raise NotImplementedError(msg)
    raise PolarNativeError(f"libpolar_mi355x error {rc}: {msg}")


def device_count() -> int:
    n = lib().pscl_device_count()
    if n < 0:
        raise PolarNativeError(last_error())
    return n


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data


def poly_value(crc) -> int:
    """The reference's CRC polynomial hex string (crc.py:10-16) as an integer (0 = no CRC)."""
    if crc is None:
        return 0
    if isinstance(crc, (int, np.integer)):
        return int(crc)
    if not crc:
        raise ValueError("CRC polynomial string must be non-empty")
    return int(str(crc), 16)


class Decoder:
    """One pscl_handle: a polar code (N, info set, list size, CRC) bound to one device."""

    def __init__(self, N: int, info_set, L: int, crc=None, device: int = 0):
        info = np.ascontiguousarray(np.asarray(info_set).astype(np.int32).ravel())
        self.N, self.K, self.L = int(N), int(info.size), int(L)
        self.info_set = info
        self.crc_poly = poly_value(crc)
        self.crc_deg = max(self.crc_poly.bit_length() - 1, 0)
        self.W = (self.K + 63) // 64 if self.K else 1
        self.device = int(device)
        h = _vp()
        check(lib().pscl_create(C.byref(h), self.device, self.N, info.ctypes.data_as(C.POINTER(_i32)), self.K,
                                self.L, self.crc_poly))
        self._hraw = h
        self._lock = threading.Lock()
        self.E = 0
        self._beta = None

    def set_rate_match(self, E: int) -> None:
        """NR: decode inputs become [B, E] received LLRs (de-rate-match + de-interleave on GPU)."""
        check(lib().pscl_set_rate_match(self._h, int(E)))
        self.E = int(E)

    @property
    def _h(self):
        h = getattr(self, "_hraw", None)
        if h is None:
            raise RuntimeError("Decoder is closed (close(), or release_decoders() on a get_decoder() handle)")
        return h

    @property
    def handle(self):
        return self._h

    @property
    def closed(self) -> bool:
        return getattr(self, "_hraw", None) is None

    def close(self) -> None:
        if getattr(self, "_hraw", None):
            lib().pscl_destroy(self._hraw)
            self._hraw = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    # ---------------------------------------------------------------- host buffers
    def decode(self, llr: np.ndarray, forced: np.ndarray | None = None, *, want_metrics=True,
               want_cands=True, want_info_llrs=True):
        """Batched decode_scl on host arrays.  llr: [B, N] float64."""
        llr = np.ascontiguousarray(llr, dtype=np.float64)
        if llr.ndim == 1:
            llr = llr[None, :]
        B = llr.shape[0]
        if llr.shape[1] != (self.E or self.N):
            raise ValueError("Channel LLR length must be a power of two" if not self.E
                             else f"expected {self.E} rate-matched LLRs per frame")
        if forced is not None:
            forced = np.ascontiguousarray(forced, dtype=np.int8).reshape(B, self.K)
        out = {
            "n_paths": np.zeros(B, np.int32),
            "best_bits": np.zeros((B, self.K), np.int8),
            "crc_pass": np.zeros(B, np.uint8),
            "best_idx": np.zeros(B, np.int32),
            "metrics": np.full((B, self.L), np.nan) if want_metrics else None,
            "cands": np.zeros((B, self.L, self.K), np.int8) if want_cands else None,
            "info_llrs": np.full((B, self.L, self.K), np.nan) if want_info_llrs else None,
        }
        with self._lock:
            check(lib().pscl_decode(self._h, _ptr(llr), B, _ptr(forced), _ptr(out["n_paths"]),
                                    _ptr(out["best_bits"]), _ptr(out["crc_pass"]), _ptr(out["best_idx"]),
                                    _ptr(out["metrics"]), _ptr(out["cands"]), _ptr(out["info_llrs"])))
        out["crc_pass"] = out["crc_pass"].astype(bool)
        return out

    def sc_decode(self, llr: np.ndarray) -> np.ndarray:
        llr = np.ascontiguousarray(llr, dtype=np.float64)
        if llr.ndim == 1:
            llr = llr[None, :]
        bits = np.zeros((llr.shape[0], self.K), np.int8)
        with self._lock:
            check(lib().pscl_sc_decode(self._h, _ptr(llr), llr.shape[0], _ptr(bits)))
        return bits

    # -------------------------------------------------------------- device buffers
    def set_stream(self, stream_ptr: int | None) -> None:
        check(lib().pscl_set_stream(self._h, stream_ptr))

    def decode_device(self, d_llr: int, B: int, *, d_force=0, d_best=0, d_flags=0, d_metrics=0, d_cands=0,
                      d_info_llrs=0, d_ref=0, k_payload=0, d_counters=0) -> None:
        check(lib().pscl_decode_device(self._h, d_llr, B, d_force or None, d_best or None, d_flags or None,
                                       d_metrics or None, d_cands or None, d_info_llrs or None, d_ref or None,
                                       int(k_payload), d_counters or None))

    def channel_device(self, seed: int, stream_id: int, ebno_db: float, rate: float, k_payload: int, frame0: int,
                       B: int, d_llr: int, d_msg: int = 0) -> None:
        check(lib().pscl_channel_device(self._h, int(seed) & (2**64 - 1), int(stream_id) & 0xFFFFFFFF,
                                        float(ebno_db), float(rate), int(k_payload), int(frame0), int(B), d_llr,
                                        d_msg or None))

    def path_llrs_device(self, d_llr: int, B: int, d_bits: int, d_out: int) -> None:
        """Decision LLRs [B, K] of the paths with information bits d_bits [B, W] (replay)."""
        with self._lock:
            check(lib().pscl_path_llrs_device(self._h, d_llr, int(B), d_bits, d_out))

    def path_llrs(self, llr: np.ndarray, bits: np.ndarray) -> np.ndarray:
        """Host form of path_llrs_device: llr [B, N] (or [B, E]), bits [B, K] 0/1."""
        llr = np.ascontiguousarray(llr, dtype=np.float64)
        if llr.ndim == 1:
            llr = llr[None, :]
        B = llr.shape[0]
        words = np.zeros((B, self.W), np.uint64)
        bits = np.asarray(bits, dtype=np.uint64).reshape(B, self.K)
        for j in range(self.K):
            words[:, j >> 6] |= bits[:, j] << np.uint64(j & 63)
        with DeviceArena(self) as mem:
            d_llr = mem.alloc(llr.nbytes)
            d_bits = mem.alloc(words.nbytes)
            d_out = mem.alloc(max(B * self.K * 8, 8))
            mem.upload(d_llr, llr)
            mem.upload(d_bits, words)
            self.path_llrs_device(d_llr, B, d_bits, d_out)
            return mem.download(d_out, B * self.K * 8, np.float64).reshape(B, self.K)

    def set_beta(self, beta: np.ndarray | None) -> None:
        """DL-SCL flip metric matrix [K, K] (None: rank by |L0|); widened to float64 exactly."""
        if beta is None:
            if self._beta is not None:
                check(lib().pscl_set_beta(self._h, None))
            self._beta = None
            return
        b = np.asarray(beta)
        if b.ndim != 2 or b.shape[0] != b.shape[1] or b.shape[0] != self.K:
            raise ValueError("beta must be a square matrix matching abs_l0 length")
        b = np.ascontiguousarray(b, dtype=np.float64)
        if self._beta is not None and np.array_equal(self._beta, b):
            return
        check(lib().pscl_set_beta(self._h, _ptr(b)))
        self._beta = b.copy()

    def dlscl_device(self, d_llr: int, B: int, retries: int, *, beta=None, d_best: int, d_flags: int,
                     d_attempts=0, d_tried=0, tried_stride=0, d_ref=0, k_payload=0, d_counters_scl=0,
                     d_counters_dl=0) -> None:
        """SCL + DL-SCL retries of B device-resident frames (pscl_dlscl_device)."""
        self.set_beta(beta)
        with self._lock:
            check(lib().pscl_dlscl_device(self._h, d_llr, int(B), int(retries), d_best, d_flags, d_attempts or None,
                                          d_tried or None, int(tried_stride), d_ref or None, int(k_payload),
                                          d_counters_scl or None, d_counters_dl or None))

    def uncoded_device(self, seed: int, stream_id: int, ebno_db: float, k_payload: int, frame0: int, B: int,
                       d_counters: int) -> None:
        check(lib().pscl_uncoded_device(self._h, int(seed) & (2**64 - 1), int(stream_id) & 0xFFFFFFFF,
                                        float(ebno_db), int(k_payload), int(frame0), int(B), d_counters))

    def sync(self) -> None:
        check(lib().pscl_sync(self._h))

    def simulate(self, seed: int, stream_id: int, ebno_db: float, rate: float, k_payload: int, frame0: int, B: int,
                 retries: int, include_uncoded: bool = False) -> np.ndarray:
        """One SNR point in one call (pscl_simulate): int64 counters [3, PSCL_NCOUNT], rows
        SCL, DL-SCL, uncoded."""
        out = np.zeros((3, PSCL_NCOUNT), np.int64)
        with self._lock:
            check(lib().pscl_simulate(self._h, int(seed) & (2**64 - 1), int(stream_id) & 0xFFFFFFFF, float(ebno_db),
                                      float(rate), int(k_payload), int(frame0), int(B), int(retries),
                                      int(bool(include_uncoded)), out.ctypes.data))
        return out

    def simulate_device(self, seed: int, stream_id: int, ebno_db: float, rate: float, k_payload: int, frame0: int,
                        B: int, retries: int, include_uncoded: bool, d_counters: int) -> None:
        """pscl_simulate enqueued, counters ADDED into device int64 [3, PSCL_NCOUNT] at d_counters
        (complete after join()/sync(); on a pipelined handle the retry chains overlap the next call)."""
        with self._lock:
            check(lib().pscl_simulate_device(self._h, int(seed) & (2**64 - 1), int(stream_id) & 0xFFFFFFFF,
                                             float(ebno_db), float(rate), int(k_payload), int(frame0), int(B),
                                             int(retries), int(bool(include_uncoded)), d_counters))

    def screening_count(self) -> int:
        """Frames the last screening decode handed to the exact re-decode (synchronizes)."""
        n = _i64()
        check(lib().pscl_screening_count(self._h, C.byref(n)))
        return int(n.value)

    def softplus_tails(self, v: np.ndarray):
        """(exact, screening) metric tails log1p(exp(-|v|)) of v as the kernels evaluate them."""
        v = np.ascontiguousarray(v, dtype=np.float64).ravel()
        with DeviceArena(self) as mem:
            d_v, d_e, d_a = mem.alloc(v.nbytes), mem.alloc(v.nbytes), mem.alloc(v.nbytes)
            mem.upload(d_v, v)
            check(lib().pscl_softplus_tails_device(self._h, d_v, v.size, d_e, d_a))
            return mem.download(d_e, v.nbytes, np.float64), mem.download(d_a, v.nbytes, np.float64)

    def tail_abs_scan(self, lo: int = 0, hi: int = 0x7F800000, bits: bool = False):
        """Largest |screening tail - exact tail| over the fp32 bit patterns [lo, hi] and the x32
        where it occurs (pscl_tail_abs_scan_device; the default range is every x32 >= 0).  bits:
        the bits form of the lane kernels' plain decodes (pscl_tail2_scan_device)."""
        fn = lib().pscl_tail2_scan_device if bits else lib().pscl_tail_abs_scan_device
        with DeviceArena(self) as mem:
            d = mem.alloc(16)
            mem.memset(d, 0, 16)
            check(fn(self._h, int(lo), int(hi), d))
            out = mem.download(d, 16, np.uint64)
        err = float(out[:1].view(np.float64)[0])
        x32 = float(np.array([int(out[1]) & 0xFFFFFFFF], np.uint32).view(np.float32)[0])
        return err, x32

    def set_pipelined(self, on: bool = True, depth: int = 2) -> None:
        """Throughput mode for streams of plain decodes (include/polar_scl.h): a screening
        decode's exact re-decode overlaps the next decode; join() / sync() order it back.  depth
        (1..4): a DL-SCL call's buffers are free again at the depth-th following call -- at the
        second at the earliest, so depth 1 behaves as 2 (a call's chains always overlap the next
        call's baseline)."""
        if not 1 <= int(depth) <= 4:
            raise ValueError(f"pipelined depth must be 1..4 (got {depth})")
        check(lib().pscl_set_pipelined(self._h, (int(depth) if depth > 2 else 1) if on else 0))

    def join(self) -> None:
        """Order pending pipelined work into the handle's stream: the plain decodes' re-decodes
        without a host wait; a pending pipelined DL-SCL call's chains are enqueued here, which
        waits on the host for that call's baseline decode (its failing-frame count)."""
        check(lib().pscl_join(self._h))

    def set_tuning(self, **knobs) -> None:
        """Schedule knobs of this handle (pscl_set_tuning; 0 = default): dl_screen, dl_chunks,
        dl_split, side_priority, post_grid, retry_wpg.  Results never depend on them."""
        for k, v in knobs.items():
            if k not in TUNE:
                raise ValueError(f"unknown tuning knob {k!r}")
            check(lib().pscl_set_tuning(self._h, TUNE[k], int(v)))
            tun = self.__dict__.setdefault("_tuning", {})
            tun[k] = int(v)

    def get_tuning(self) -> dict:
        """The knobs set on this handle through set_tuning (0 = default for any other knob)."""
        return dict(self.__dict__.get("_tuning", {}))

    def set_screening(self, on: bool = True) -> None:
        """Screening decode for plain decodes (default on; include/polar_scl.h)."""
        check(lib().pscl_set_screening(self._h, 1 if on else 0))

    def timing_enable(self, on: bool = True) -> None:
        check(lib().pscl_timing_enable(self._h, 1 if on else 0))

    def timing_read(self):
        n, ms = _i64(), _dbl()
        check(lib().pscl_timing_read(self._h, C.byref(n), C.byref(ms)))
        return int(n.value), float(ms.value)

    def timing_read_split(self):
        """((launches, ms) on the handle's stream, (launches, ms) on its side streams)."""
        n0, t0, n1, t1 = _i64(), _dbl(), _i64(), _dbl()
        check(lib().pscl_timing_read_split(self._h, C.byref(n0), C.byref(t0), C.byref(n1), C.byref(t1)))
        return (int(n0.value), float(t0.value)), (int(n1.value), float(t1.value))

    def host_stats(self, reset: bool = False):
        """(call ms, wait ms, calls) of the DL-SCL calls on the host (pscl_host_stats)."""
        c, w, n = _dbl(), _dbl(), _i64()
        check(lib().pscl_host_stats(self._h, C.byref(c), C.byref(w), C.byref(n), 1 if reset else 0))
        return float(c.value), float(w.value), int(n.value)

    def path_stats(self) -> dict:
        """Schedules enqueued so far (pscl_path_stats): fused-post rounds, separate-post rounds,
        fused-TX blocks, 4-entry-form post launches, exact lane-per-path launches."""
        a, b, c, d, x = _i64(), _i64(), _i64(), _i64(), _i64()
        check(lib().pscl_path_stats(self._h, C.byref(a), C.byref(b), C.byref(c), C.byref(d), C.byref(x)))
        return {"fused_post_rounds": int(a.value), "post_rounds": int(b.value), "fused_tx_blocks": int(c.value),
                "post_epw4_launches": int(d.value), "lane_exact_launches": int(x.value)}

    def launch_info(self, B: int):
        w, g, lds = C.c_int(), _i64(), C.c_int()
        check(lib().pscl_launch_info(self._h, int(B), C.byref(w), C.byref(g), C.byref(lds)))
        return int(w.value), int(g.value), int(lds.value)


class CpuDecoder:
    """The product's host decoder (pscl_decode_cpu): Decoder.decode's contract and outputs, bit for
    bit, with no GPU -- the reference's CPU-only runs (BASELINE config 1).  device = "cpu"."""

    def __init__(self, N: int, info_set, L: int, crc=None, threads: int = 0):
        info = np.ascontiguousarray(np.asarray(info_set).astype(np.int32).ravel())
        self.N, self.K, self.L = int(N), int(info.size), int(L)
        self.info_set = info
        self.crc_poly = poly_value(crc)
        self.crc_deg = max(self.crc_poly.bit_length() - 1, 0)
        self.W = (self.K + 63) // 64 if self.K else 1
        self.E = 0
        self.device = "cpu"
        self.threads = int(threads or os.environ.get("PSCL_CPU_THREADS", "0") or 0)
        if self.N < 2 or self.N & (self.N - 1) or self.N > PSCL_MAX_N:
            raise ValueError("Channel LLR length must be a power of two")
        if self.crc_poly and self.K <= self.crc_deg:
            raise ValueError("Message too short for the provided CRC polynomial")

    def decode(self, llr: np.ndarray, forced: np.ndarray | None = None, *, want_metrics=True,
               want_cands=True, want_info_llrs=True):
        llr = np.ascontiguousarray(llr, dtype=np.float64)
        if llr.ndim == 1:
            llr = llr[None, :]
        B = llr.shape[0]
        if llr.shape[1] != self.N:
            raise ValueError("Channel LLR length must be a power of two")
        if forced is not None:
            forced = np.ascontiguousarray(forced, dtype=np.int8).reshape(B, self.K)
            if np.any((forced < -1) | (forced > 1)):
                raise ValueError("force_info_bits entries must be -1, 0, or 1")
        out = {
            "n_paths": np.zeros(B, np.int32),
            "best_bits": np.zeros((B, self.K), np.int8),
            "crc_pass": np.zeros(B, np.uint8),
            "best_idx": np.zeros(B, np.int32),
            "metrics": np.full((B, self.L), np.nan) if want_metrics else None,
            "cands": np.zeros((B, self.L, self.K), np.int8) if want_cands else None,
            "info_llrs": np.full((B, self.L, self.K), np.nan) if want_info_llrs else None,
        }
        check(lib().pscl_decode_cpu(self.N, self.info_set.ctypes.data_as(C.POINTER(_i32)), self.K, self.L,
                                    self.crc_poly, _ptr(llr), B, _ptr(forced), _ptr(out["n_paths"]),
                                    _ptr(out["best_bits"]), _ptr(out["crc_pass"]), _ptr(out["best_idx"]),
                                    _ptr(out["metrics"]), _ptr(out["cands"]), _ptr(out["info_llrs"]), self.threads))
        out["crc_pass"] = out["crc_pass"].astype(bool)
        return out

    def sync(self) -> None:
        pass

    def close(self) -> None:
        pass


_CACHE: dict = {}
_CACHE_LOCK = threading.Lock()


def get_decoder(N: int, info_set, L: int, crc=None, device: int = 0, E: int = 0, slot: int = 0) -> Decoder:
    """Cached Decoder per (N, info set, L, CRC, device, rate-matched length E, slot).  Distinct
    slots are distinct handles (own streams and scratch), for concurrent host threads."""
    info = np.asarray(info_set).astype(np.int64).ravel()
    cpu = isinstance(device, str) and device == "cpu"
    key = (int(N), info.tobytes(), int(L), poly_value(crc), "cpu" if cpu else int(device), int(E), int(slot))
    with _CACHE_LOCK:
        dec = _CACHE.get(key)
        if dec is None:
            if len(_CACHE) > 64:
                _CACHE.clear()
            if cpu:
                if E:
                    raise NotImplementedError("the CPU decoder takes internal (de-rate-matched) LLRs")
                dec = _CACHE[key] = CpuDecoder(N, info, L, crc)
                return dec
            dec = Decoder(N, info, L, crc, device)
            if E:
                dec.set_rate_match(E)
            _CACHE[key] = dec
        return dec


def release_decoders() -> None:
    """Close every cached decoder (get_decoder): their handles, streams and device scratch go.  A
    long-lived process that is done with a workload calls this so that the next one's streams are
    not spread over hardware queues shared with idle ones.  Every Decoder an earlier get_decoder()
    returned is closed too (flip.decode_with_retries_device and the sweeps share them): using one
    afterwards raises RuntimeError; call get_decoder() again for a fresh handle."""
    with _CACHE_LOCK:
        decs = list(_CACHE.values())
        _CACHE.clear()
    for d in decs:
        d.close()


class DeviceArena:
    """Device buffers owned through the C ABI (pscl_device_alloc), freed on exit.  Lets the
    host layer drive the device path without PyTorch."""

    def __init__(self, dec: Decoder):
        self.dec = dec
        self.ptrs: list[int] = []

    def __enter__(self) -> "DeviceArena":
        return self

    def __exit__(self, *exc) -> None:
        self.dec.sync()
        for p in self.ptrs:
            lib().pscl_device_free(self.dec.handle, p)
        self.ptrs.clear()

    def alloc(self, nbytes: int) -> int:
        p = _vp()
        check(lib().pscl_device_alloc(self.dec.handle, C.byref(p), int(nbytes)))
        self.ptrs.append(p.value)
        return p.value

    def memset(self, d_ptr: int, value: int, nbytes: int) -> None:
        check(lib().pscl_memset_device(self.dec.handle, d_ptr, int(value), int(nbytes)))

    def upload(self, d_ptr: int, arr: np.ndarray) -> None:
        arr = np.ascontiguousarray(arr)
        check(lib().pscl_memcpy_htod(self.dec.handle, d_ptr, arr.ctypes.data, arr.nbytes))

    def download(self, d_ptr: int, nbytes: int, dtype) -> np.ndarray:
        out = np.empty(int(nbytes) // np.dtype(dtype).itemsize, dtype=dtype)
        check(lib().pscl_memcpy_dtoh(self.dec.handle, out.ctypes.data, d_ptr, out.nbytes))
        return out
