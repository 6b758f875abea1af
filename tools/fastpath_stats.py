"""How often the decoder's exact fast paths fire (diagnostic build with -DPSCL_STATS).

    PSCL_LIB_PATH=tools/_variant/lib_stats.so python tools/fastpath_stats.py [L] [ebno]
Counters (per wavefront): [8] frozen phases, [9] frozen re-ranks skipped, [10] info phases on
the full ranking path, [11] info phases kept in place (exact kernel); [12..15] screening
full-list info phases by the wave's worst frame: 0, 1, 2, >= 3 worse children within the
margin of the largest better child.
"""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from polar_code_amd import _native  # noqa: E402
from polar_code_amd.polar.polar import construct_info_set  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ebno = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
B = 200_000
dec = _native.Decoder(128, construct_info_set(128, 64), L, "0x1864CFB")
dec.set_stream(torch.cuda.current_stream().cuda_stream)
llr = torch.empty((B, 128), dtype=torch.float64, device="cuda")
msg = torch.empty((B, 1), dtype=torch.int64, device="cuda")
best = torch.empty((B, 1), dtype=torch.int64, device="cuda")
cnt = torch.zeros(64, dtype=torch.int64, device="cuda")  # the stats builds write slots 8..42
dec.channel_device(0, int(ebno * 10), ebno, 0.5, 40, 0, B, llr.data_ptr(), msg.data_ptr())
dec.decode_device(llr.data_ptr(), B, d_best=best.data_ptr(), d_ref=msg.data_ptr(), k_payload=40,
                  d_counters=cnt.data_ptr())
torch.cuda.synchronize()
c = cnt.cpu().tolist()
print(f"L={L} {ebno} dB: frozen {c[8]} skipped {c[9]} ({c[9] / max(c[8], 1):.1%}); info full {c[10]} "
      f"kept {c[11]} ({c[11] / max(c[10] + c[11], 1):.1%}); FER {c[1] / B:.4f}")
tot = max(sum(c[12:16]), 1)
if os.environ.get("PSCL_LANE_STATS"):  # the lane-per-path kernel's tiers (scl128_lane.hip)
    print("lane kernel full-list info phases (waves): " +
          ", ".join(f"{k}: {c[12 + i]} ({c[12 + i] / tot:.1%})" for i, k in enumerate(["kept", "one swap", "ranked"])))
    if sum(c[16:25]):  # PSCL_STATS=2: the ranked tier's frames and waves
        def hist(a):
            t = max(sum(a), 1)
            return ", ".join(f"{i}: {v} ({v / t:.1%})" for i, v in enumerate(a) if v)
        print("ranked-tier frames by surviving worse children d: " + hist(c[16:25]))
        print("ranked-tier frames by near-worse children: " + hist(c[25:34]))
        print("ranked-tier waves by the largest d of their frames: " + hist(c[34:43]))
else:
    print("screening full-list info phases (waves) by worst frame's near-worse children: " +
          ", ".join(f"{k}: {c[12 + i]} ({c[12 + i] / tot:.1%})" for i, k in enumerate(["0", "1", "2", ">=3"])))
