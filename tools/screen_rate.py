"""Fraction of frames the screening decode hands to the exact re-decode, per list size and
Eb/N0 (Philox channel, P(128,64)+CRC-24; NR (128,88) E=256 with --nr).

    python tools/screen_rate.py [B]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from polar_code_amd import _native  # noqa: E402
from polar_code_amd.polar.polar import construct_info_set  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
for E, K in ((0, 64), (256, 88)):
    info = construct_info_set(128, K)
    for L in (8, 4, 2, 1):
        dec = _native.Decoder(128, info, L, "0x1864CFB")
        if E:
            dec.set_rate_match(E)
        n_in = E or 128
        with _native.DeviceArena(dec) as mem:
            d_llr, d_msg = mem.alloc(B * n_in * 8), mem.alloc(B * 16)
            d_best, d_flags = mem.alloc(B * 16), mem.alloc(B)
            for eb in (3.0, 4.0, 5.0, 6.0):
                rate = (K - 24) / E if E else K / 128
                dec.channel_device(0, int(eb * 10), eb, rate, K - 24, 0, B, d_llr, d_msg)
                dec.decode_device(d_llr, B, d_best=d_best, d_flags=d_flags)
                n = dec.screening_count()
                print(f"E={E or 128} L={L} Eb/N0={eb}: {n} of {B} frames re-decoded ({n / B:.5f})", flush=True)
        dec.close()
