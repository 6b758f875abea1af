import os, sys
sys.path.insert(0, '.')
import numpy as np
from polar_code_amd import _native
from polar_code_amd.polar.polar import construct_info_set
info = construct_info_set(128, 64)
dec = _native.Decoder(128, info, 8, "0x1864CFB")
B = 4
with _native.DeviceArena(dec) as mem:
    d_llr, d_msg = mem.alloc(B * 128 * 8), mem.alloc(B * 16)
    d_best, d_flags = mem.alloc(B * 16), mem.alloc(B)
    dec.channel_device(0, 50, 5.0, 0.5, 40, 0, B, d_llr, d_msg)
    dec.decode_device(d_llr, B, d_best=d_best, d_flags=d_flags)
    print("count", dec.screening_count(), flush=True)
