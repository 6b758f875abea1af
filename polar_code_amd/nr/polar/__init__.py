"""NR polar helpers (mirror of dl_scl_polar/nr/polar/__init__.py)."""
from .interleaver import subblock_interleave, subblock_deinterleave
from .rate_match import rate_match_polar, derate_match_polar
from .scl_nr import encode_rate_matched, decode_rate_matched_scl

__all__ = [
    "subblock_interleave",
    "subblock_deinterleave",
    "rate_match_polar",
    "derate_match_polar",
    "encode_rate_matched",
    "decode_rate_matched_scl",
]
