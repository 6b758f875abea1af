"""Throughput of the long-code decoders (csrc/scl_lane_long.hip screening + scl_long.hip exact
re-decode; L = 32: scl_long.hip alone), N = 256..1024, on one GPU.

    python tools/long_bench.py            (GPU box)
Frames: random BPSK/AWGN codewords of construct_info_set(N, K) + CRC-24 at an Eb/N0 in each
code's waterfall (the reference's construction, design SNR 2.5 dB: oracle FER at L = 8 is 0.21
for N = 256 at 4 dB, 0.32 for N = 512 at 5 dB, 0.42 for N = 1024 at 6 dB), generated on the
host once and kept resident; each timed step decodes B frames (decode_device, best bits
and flags only) on the handle's stream, timed with events on that stream.

    python tools/long_bench.py --dl       (the long-code DL-SCL loop and TX chain instead)
DL-SCL (8 flips, no beta) on device-resident frames: the device loop (pscl_dlscl_device, HIST
long-kernel retry decodes) against the host-ranked form (decode_with_retries_batch: GPU decodes
from host buffers, numpy ranking), and the device TX chain (pscl_channel_device).
"""
import time
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from polar_code_amd import _native  # noqa: E402
from polar_code_amd.polar.crc import attach_crc  # noqa: E402
from polar_code_amd.polar.polar import _polar_transform, construct_info_set  # noqa: E402

POLY = "0x1864CFB"


def dl_bench():
    from polar_code_amd.dlscl.flip import decode_with_retries_batch

    for N, K, L, B, snr in [(256, 128, 4, 50_000, 3.5), (512, 256, 4, 20_000, 4.0)]:
        rng = np.random.default_rng(N + L)
        info = construct_info_set(N, K)
        msg = attach_crc(rng.integers(0, 2, size=(B, K - 24), dtype=np.int8), POLY)
        u = np.zeros((B, N), np.int8)
        u[:, info] = msg
        nv = 1.0 / (2.0 * K / N * 10 ** (snr / 10))
        llr = 2.0 * ((1.0 - 2.0 * _polar_transform(u)) + rng.normal(0.0, np.sqrt(nv), size=(B, N))) / nv
        dec = _native.Decoder(N, info, L, POLY)
        stream = torch.cuda.Stream()
        dec.set_stream(stream.cuda_stream)
        d_llr = torch.from_numpy(llr).cuda()
        W = dec.W
        best = torch.empty((B, W), dtype=torch.int64, device="cuda")
        flags = torch.empty(B, dtype=torch.uint8, device="cuda")
        att = torch.empty(B, dtype=torch.int32, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for rep in range(2):  # (the first call sizes the state)
            e0.record(stream)
            dec.dlscl_device(d_llr.data_ptr(), B, 8, d_best=best.data_ptr(), d_flags=flags.data_ptr(),
                             d_attempts=att.data_ptr())
            e1.record(stream)
            torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        a = att.cpu().numpy()
        t0 = time.perf_counter()
        host = decode_with_retries_batch(llr, info, L, 8, crc=POLY)
        hs = time.perf_counter() - t0
        same = bool((host["attempts"] == a).all())
        d_msg = torch.empty((B, W), dtype=torch.int64, device="cuda")
        dec.channel_device(1, 35, snr, K / N, K - 24, 0, B, d_llr.data_ptr(), d_msg.data_ptr())
        torch.cuda.synchronize()
        e0.record(stream)
        dec.channel_device(1, 35, snr, K / N, K - 24, 0, B, d_llr.data_ptr(), d_msg.data_ptr())
        e1.record(stream)
        torch.cuda.synchronize()
        tx = e0.elapsed_time(e1)
        print(f"N={N} K={K} L={L} {snr:g} dB, {B} frames: DL-SCL device loop {B / ms * 1e3 / 1e6:.3f} M frames/s "
              f"({ms:.1f} ms; {int((a > 1).sum())} frames retried, {int(a.sum() - B)} re-decodes); host-ranked "
              f"form {B / hs / 1e6:.3f} M frames/s ({hs * 1e3:.0f} ms), attempts equal: {same}; TX chain "
              f"{B / tx * 1e3 / 1e6:.1f} M frames/s", flush=True)
        dec.close()


if "--dl" in sys.argv:
    dl_bench()
    sys.exit(0)
# (N = 128, K = 100, and every L = 16 / 32 decode: the runtime-information-set lane kernel -- no
# compiled-in screening kernel -- timed against the exact kernel alone too)
CASES = [(128, 100, 8, 500_000, 4.5), (256, 128, 8, 200_000, 4.0), (512, 256, 8, 100_000, 5.0),
         (1024, 512, 8, 50_000, 6.0), (128, 64, 16, 200_000, 4.0), (256, 128, 16, 100_000, 4.0),
         (1024, 512, 16, 20_000, 6.0), (128, 64, 32, 100_000, 4.0), (1024, 512, 32, 20_000, 6.0)]
# --big: the N = 1024 rows at 4x the batch (the 50 000-frame batch at L = 8 is 6.1 waves per SIMD
# slot: its last wave round runs a tenth full)
if "--big" in sys.argv:
    CASES = [(1024, 512, 8, 200_000, 6.0), (1024, 512, 16, 80_000, 6.0), (1024, 512, 32, 80_000, 6.0)]
for N, K, L, B, snr in CASES:
    rng = np.random.default_rng(N + L)
    info = construct_info_set(N, K)
    msg = attach_crc(rng.integers(0, 2, size=(B, K - 24), dtype=np.int8), POLY)
    u = np.zeros((B, N), np.int8)
    u[:, info] = msg
    nv = 1.0 / (2.0 * K / N * 10 ** (snr / 10))
    llr = 2.0 * ((1.0 - 2.0 * _polar_transform(u)) + rng.normal(0.0, np.sqrt(nv), size=(B, N))) / nv
    dec = _native.Decoder(N, info, L, POLY)
    stream = torch.cuda.Stream()  # (not the legacy default stream: its handle is 0)
    dec.set_stream(stream.cuda_stream)
    d_llr = torch.from_numpy(llr).cuda()
    best = torch.empty((B, dec.W), dtype=torch.int64, device="cuda")
    flags = torch.empty(B, dtype=torch.uint8, device="cuda")
    best2 = torch.empty_like(best)
    flags2 = torch.empty_like(flags)
    dec.decode_device(d_llr.data_ptr(), B, d_best=best.data_ptr(), d_flags=flags.data_ptr())
    torch.cuda.synchronize()
    n_def = dec.screening_count()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    steps = 3
    e0.record(stream)
    for _ in range(steps):
        dec.decode_device(d_llr.data_ptr(), B, d_best=best.data_ptr(), d_flags=flags.data_ptr())
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    fer = float(((flags.cpu().numpy() & 0x80) == 0).mean())
    exact_note = ""
    if N == 128 or L >= 16:  # the same decode on the exact kernel alone (screening off)
        dec.set_screening(False)
        e0.record(stream)
        for _ in range(steps):
            dec.decode_device(d_llr.data_ptr(), B, d_best=best2.data_ptr(), d_flags=flags2.data_ptr())
        e1.record(stream)
        torch.cuda.synchronize()
        exact_note = (f", exact kernel alone {B / (e0.elapsed_time(e1) / steps) * 1e3 / 1e6:.2f} M frames/s "
                      f"(outputs equal {bool(torch.equal(best, best2) and torch.equal(flags, flags2))})")
        dec.set_screening(True)
    # pipelined handle (as bench.py): each call's exact re-decode of its deferred frames overlaps
    # the next call's screening pass; alternating output buffers, the last re-decode inside the
    # timed region (join)
    dec.set_pipelined(True)
    outs = [(best, flags), (best2, flags2)]
    for i in range(2):
        dec.decode_device(d_llr.data_ptr(), B, d_best=outs[i][0].data_ptr(), d_flags=outs[i][1].data_ptr())
    dec.join()
    torch.cuda.synchronize()
    psteps = 6
    e0.record(stream)
    for i in range(psteps):
        dec.decode_device(d_llr.data_ptr(), B, d_best=outs[i & 1][0].data_ptr(), d_flags=outs[i & 1][1].data_ptr())
    dec.join()
    e1.record(stream)
    torch.cuda.synchronize()
    pms = e0.elapsed_time(e1) / psteps
    same = bool(torch.equal(best, best2) and torch.equal(flags, flags2))
    print(f"N={N} K={K} L={L} {snr:g} dB: {B / ms * 1e3 / 1e6:.2f} M frames/s ({ms:.2f} ms per {B} frames), "
          f"pipelined {B / pms * 1e3 / 1e6:.2f} M frames/s ({pms:.2f} ms), input {B * N * 8 / pms / 1e6:.1f} GB/s, "
          f"FER {fer:.4f}, deferred to the exact kernel {n_def} ({100.0 * n_def / B:.2f} %), outputs equal {same}"
          f"{exact_note}",
          flush=True)
    dec.close()
