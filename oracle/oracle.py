"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/liboracle_scl.so (the C restatement of the reference,
oracle/scl_oracle.c).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import this module; polar_code_amd never does.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB = None


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        path = _HERE / "liboracle_scl.so"
        if not path.exists():
            raise RuntimeError(f"{path} missing: run python -m polar_code_amd.build")
        L = C.CDLL(str(path))
        dp, ip, bp = C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_int8)
        L.oracle_attach_crc.argtypes = [bp, C.c_int, C.c_uint64, bp]
        L.oracle_check_crc.argtypes = [bp, C.c_int, C.c_uint64]
        L.oracle_polar_transform.argtypes = [bp, C.c_int]
        L.oracle_construct_info_set.argtypes = [C.c_int, C.c_int, C.c_double, ip]
        L.oracle_sc_decode.argtypes = [dp, C.c_int, ip, C.c_int, bp]
        L.oracle_decode_scl.argtypes = [dp, C.c_int, ip, C.c_int, C.c_int, C.c_uint64, bp, bp, dp, dp, ip]
        L.oracle_decode_with_retries.argtypes = [dp, C.c_int, ip, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                                 C.POINTER(C.c_float), bp, ip, ip, ip, ip]
        L.oracle_decode_batch.argtypes = [dp, C.c_int64, C.c_int, ip, C.c_int, C.c_int, C.c_uint64, bp,
                                          C.POINTER(C.c_uint8), ip]
        L.oracle_dl_batch.argtypes = [dp, C.c_int64, C.c_int, ip, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                      C.POINTER(C.c_float), bp, ip, ip]
        L.oracle_num_threads.restype = C.c_int
        L.oracle_set_num_threads.argtypes = [C.c_int]
        L.oracle_logaddexp0_batch.argtypes = [dp, C.c_int64, dp]
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def poly_int(crc) -> int:
    return 0 if crc is None or crc == "" else int(str(crc), 16)


def attach_crc(msg, crc):
    msg = np.ascontiguousarray(msg, np.int8)
    deg = poly_int(crc).bit_length() - 1
    out = np.zeros(msg.size + deg, np.int8)
    lib().oracle_attach_crc(_p(msg, C.c_int8), msg.size, poly_int(crc), _p(out, C.c_int8))
    return out


def check_crc(msg, crc) -> bool:
    msg = np.ascontiguousarray(msg, np.int8)
    r = lib().oracle_check_crc(_p(msg, C.c_int8), msg.size, poly_int(crc))
    if r < 0:
        raise ValueError("Message too short for the provided CRC polynomial")
    return bool(r)


def polar_transform(u):
    x = np.ascontiguousarray(u, np.int8).copy()
    lib().oracle_polar_transform(_p(x, C.c_int8), x.size)
    return x


def construct_info_set(N, K, design_snr_db=2.5):
    out = np.zeros(K, np.int32)
    if lib().oracle_construct_info_set(N, K, design_snr_db, _p(out, C.c_int32)):
        raise ValueError("bad N/K")
    return out


def sc_decode(llr, info):
    llr = np.ascontiguousarray(llr, np.float64)
    info = np.ascontiguousarray(info, np.int32)
    out = np.zeros(info.size, np.int8)
    if lib().oracle_sc_decode(_p(llr, C.c_double), llr.size, _p(info, C.c_int32), info.size, _p(out, C.c_int8)):
        raise ValueError("bad input")
    return out


def decode_scl(llr, info, M, crc=None, force=None):
    """Returns (n_paths, cands[M,K], metrics[M], info_llrs[M,K], best_index)."""
    llr = np.ascontiguousarray(llr, np.float64)
    info = np.ascontiguousarray(info, np.int32)
    K = info.size
    cands = np.zeros((M, K), np.int8)
    mets = np.full(M, np.nan)
    illr = np.full((M, K), np.nan)
    best = np.zeros(1, np.int32)
    fp = None
    if force is not None:
        force = np.ascontiguousarray(force, np.int8)
        fp = _p(force, C.c_int8)
    n = lib().oracle_decode_scl(_p(llr, C.c_double), llr.size, _p(info, C.c_int32), K, M, poly_int(crc), fp,
                                _p(cands, C.c_int8), _p(mets, C.c_double), _p(illr, C.c_double),
                                _p(best, C.c_int32))
    if n < 0:
        raise ValueError(f"oracle_decode_scl error {n}")
    return n, cands, mets, illr, int(best[0])


def decode_with_retries(llr, info, M, retries, crc=None, beta=None):
    """Returns dict(bits, success, attempts, tried)."""
    llr = np.ascontiguousarray(llr, np.float64)
    info = np.ascontiguousarray(info, np.int32)
    K = info.size
    bits = np.zeros(K, np.int8)
    succ, att, nt = (np.zeros(1, np.int32) for _ in range(3))
    tried = np.full(max(retries, 1), -1, np.int32)
    bp = None
    if beta is not None:
        beta = np.ascontiguousarray(beta, np.float32)
        bp = _p(beta, C.c_float)
    rc = lib().oracle_decode_with_retries(_p(llr, C.c_double), llr.size, _p(info, C.c_int32), K, M, retries,
                                          poly_int(crc), bp, _p(bits, C.c_int8), _p(succ, C.c_int32),
                                          _p(att, C.c_int32), _p(tried, C.c_int32), _p(nt, C.c_int32))
    if rc:
        raise ValueError(f"oracle_decode_with_retries error {rc}")
    return dict(bits=bits, success=bool(succ[0]), attempts=int(att[0]), tried=tried[: nt[0]].tolist())


def decode_batch(llr, info, M, crc=None, want_idx=False):
    """Parallel (OpenMP) batch decode: returns (best_bits[B,K], crc_pass[B]) and, with
    want_idx, best_index[B] (the best candidate's list position) as a third element."""
    llr = np.ascontiguousarray(llr, np.float64)
    info = np.ascontiguousarray(info, np.int32)
    B, N = llr.shape
    K = info.size
    bits = np.zeros((B, K), np.int8)
    ok = np.zeros(B, np.uint8)
    idx = np.zeros(B, np.int32) if want_idx else None
    if lib().oracle_decode_batch(_p(llr, C.c_double), B, N, _p(info, C.c_int32), K, M, poly_int(crc),
                                 _p(bits, C.c_int8), _p(ok, C.c_uint8), None if idx is None else _p(idx, C.c_int32)):
        raise ValueError("oracle_decode_batch failed")
    return (bits, ok.astype(bool), idx) if want_idx else (bits, ok.astype(bool))


def dl_batch(llr, info, M, retries, crc=None, beta=None):
    """Parallel (OpenMP) decode_with_retries: returns (bits[B,K], success[B], attempts[B])."""
    llr = np.ascontiguousarray(llr, np.float64)
    info = np.ascontiguousarray(info, np.int32)
    B, N = llr.shape
    K = info.size
    bits = np.zeros((B, K), np.int8)
    succ = np.zeros(B, np.int32)
    att = np.zeros(B, np.int32)
    bp = None
    if beta is not None:
        beta = np.ascontiguousarray(beta, np.float32)
        bp = _p(beta, C.c_float)
    if lib().oracle_dl_batch(_p(llr, C.c_double), B, N, _p(info, C.c_int32), K, M, retries, poly_int(crc), bp,
                             _p(bits, C.c_int8), _p(succ, C.c_int32), _p(att, C.c_int32)):
        raise ValueError("oracle_dl_batch failed")
    return bits, succ.astype(bool), att


def num_threads() -> int:
    return int(lib().oracle_num_threads())


def set_num_threads(n: int) -> None:
    """OpenMP thread count of decode_batch / dl_batch (n > 0)."""
    lib().oracle_set_num_threads(int(n))


def logaddexp0(v):
    v = np.ascontiguousarray(v, np.float64)
    out = np.empty_like(v)
    lib().oracle_logaddexp0_batch(_p(v, C.c_double), v.size, _p(out, C.c_double))
    return out
