import sys, numpy as np
order = sys.argv[1]
if order == "torch_first":
    import torch; print("torch avail", torch.cuda.is_available())
sys.path.insert(0, ".")
from polar_code_amd import _native
from polar_code_amd.polar.polar import construct_info_set
d = _native.Decoder(128, construct_info_set(128,64), 8, "0x1864CFB")
out = d.decode(np.random.default_rng(0).normal(4, 3, (16,128)))
print("decode ok", out["crc_pass"].sum())
import torch
print("torch avail after", torch.cuda.is_available(), torch.cuda.device_count())
t = torch.zeros(10, device="cuda"); print("alloc ok", t.sum().item())
import ctypes
print([l for l in open("/proc/self/maps").read().split("\n") if "amdhip64" in l][:3])
