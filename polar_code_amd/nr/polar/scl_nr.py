"""Rate-matched polar SCL (mirror of dl_scl_polar/nr/polar/scl_nr.py).

decode_rate_matched_scl runs on the GPU: the decoder handle is configured for the received
length E and de-rate-matches + de-interleaves inside the decode kernel."""
from __future__ import annotations

from typing import Dict

import numpy as np

from ... import _native
from ...polar.crc import attach_crc
from ...polar.polar import _polar_transform
from .interleaver import subblock_interleave
from .rate_match import rate_match_polar


def _polar_encode(info_bits: np.ndarray, info_set: np.ndarray, N: int) -> np.ndarray:
    u = np.zeros(N, dtype=np.int8)
    u[info_set] = info_bits
    return _polar_transform(u)


def encode_rate_matched(payload_bits, crc_poly, N, E, info_set, ilv_mode="default") -> np.ndarray:
    """scl_nr.py:23-35: CRC attach -> polar encode -> sub-block interleave -> rate match."""
    msg = attach_crc(payload_bits, crc_poly)
    codeword = _polar_encode(msg, info_set, N)
    return rate_match_polar(subblock_interleave(codeword, mode=ilv_mode), E)


def decode_rate_matched_scl(llr_E, crc_poly, N, E, info_set, M, ilv_mode="default", *, device: int = 0) -> Dict:
    """scl_nr.py:38-57 on the GPU.  llr_E: [E] (or a batch [B, E]).  Returns payload
    (= best_path_bits[:len(info_set)]), crc_pass and best_path_bits (batched: arrays)."""
    llr_E = np.asarray(llr_E, dtype=np.float64)
    single = llr_E.ndim == 1
    if single:
        llr_E = llr_E[None, :]
    if llr_E.shape[1] != E:
        raise ValueError("llr_E length must equal E")
    dec = _native.get_decoder(N, info_set, M, crc_poly, device, E=E)
    out = dec.decode(llr_E, want_metrics=False, want_cands=False, want_info_llrs=False)
    bits = out["best_bits"]
    crc_pass = out["crc_pass"] if crc_poly else np.ones(bits.shape[0], bool)
    if single:
        return {"payload": bits[0][: len(info_set)], "crc_pass": bool(crc_pass[0]), "best_path_bits": bits[0]}
    return {"payload": bits[:, : len(info_set)], "crc_pass": crc_pass, "best_path_bits": bits}


__all__ = ["encode_rate_matched", "decode_rate_matched_scl"]
