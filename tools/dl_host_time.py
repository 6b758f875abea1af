"""Host time of pipelined DL-SCL calls (config 4: L = 4, 8 flips, beta_M4, 10^6 frames per call):
wall time of each pscl_dlscl_device call on the host against the GPU step time, to tell a
launch-bound pipeline (host time per call >= step time) from a GPU-bound one.

    python tools/dl_host_time.py [depth] [steps] [sync]   (sync: join + synchronize before each call,
                                                           so a call's host time is its enqueue cost alone)
"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from polar_code_amd import _native  # noqa: E402
from polar_code_amd.polar.polar import construct_info_set  # noqa: E402

depth = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B, L, steps = 1_000_000, 4, int(sys.argv[2]) if len(sys.argv) > 2 else 12
dec = _native.Decoder(128, construct_info_set(128, 64), L, "0x1864CFB")
dec.set_stream(torch.cuda.current_stream().cuda_stream)
dec.set_pipelined(True, depth=depth)
beta = np.load(Path(__file__).resolve().parent.parent / "tests" / "golden" / "beta_M4.npy")
llr = [torch.empty((B, 128), dtype=torch.float64, device="cuda") for _ in range(4)]
msg = [torch.empty((B, 1), dtype=torch.int64, device="cuda") for _ in range(4)]
for i in range(4):
    dec.channel_device(0, 50, 5.0, 0.5, 40, i * B, B, llr[i].data_ptr(), msg[i].data_ptr())
best = [torch.empty((B, 1), dtype=torch.int64, device="cuda") for _ in range(depth)]
flags = [torch.empty((B,), dtype=torch.uint8, device="cuda") for _ in range(depth)]
cs = torch.zeros(8, dtype=torch.int64, device="cuda")
cd = torch.zeros(8, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
ht, jt = [], []
t0 = time.perf_counter()
sync_each = len(sys.argv) > 3 and sys.argv[3] == "sync"  # pure enqueue cost: the GPU idle at each call
for s in range(steps):
    if sync_each:
        dec.join()
        torch.cuda.synchronize()
    a = time.perf_counter()
    dec.dlscl_device(llr[s % 4].data_ptr(), B, 8, beta=beta, d_best=best[s % depth].data_ptr(),
                     d_flags=flags[s % depth].data_ptr(), d_ref=msg[s % 4].data_ptr(), k_payload=40,
                     d_counters_scl=cs.data_ptr(), d_counters_dl=cd.data_ptr())
    ht.append((time.perf_counter() - a) * 1e3)
    if sync_each:  # the call's chains, enqueued by join() once its baseline has ended
        torch.cuda.synchronize()
        a = time.perf_counter()
        dec.join()
        jt.append((time.perf_counter() - a) * 1e3)
dec.join()
torch.cuda.synchronize()
tot = (time.perf_counter() - t0) * 1e3
print(f"depth {depth}: {tot / steps:.3f} ms per step; host ms per call: " + " ".join(f"{x:.2f}" for x in ht))
cm, wm, nc = dec.host_stats()
print(f"pscl_host_stats: {nc} calls, {cm / max(nc, 1):.3f} ms per call on the host, of which {wm / max(nc, 1):.3f} ms "
      f"blocked (busy {(cm - wm) / max(nc, 1):.3f} ms)")
if sync_each:
    print("join (chain enqueue) ms per call: " + " ".join(f"{x:.2f}" for x in jt))
