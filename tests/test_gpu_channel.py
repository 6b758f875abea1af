"""The on-device TX chain (pscl_channel_device) against a NumPy restatement of its stream.

Payload bits, CRC, codeword and message words must match exactly.  The Box-Muller pairs are
computed in fp32 with the hardware transcendentals (v_log_f32, v_sqrt_f32, v_sin/cos_f32, in
csrc/scl_kernels.hip bm_pair) and widened to fp64; the host restates them with numpy float32
libm calls, so the normals agree to ~1e-6 (tolerance stated in each test), with every
systematic slip (range, scaling, pairing) far outside it.  Covers plain N=128,
short codes, K > 64 (two message words), NR rate matching (repetition and puncturing) and the
long codes (N = 256..1024: channel_long_kernel, payloads beyond one Philox block).
"""
import numpy as np
import pytest

from polar_code_amd import _native
from polar_code_amd.nr.polar.interleaver import _order
from polar_code_amd.polar.crc import attach_crc
from polar_code_amd.polar.polar import construct_info_set

pytestmark = pytest.mark.gpu

M32 = np.uint64(0xFFFFFFFF)


def philox4x32(c, k0, k1):
    """Philox4x32-10 on arrays of counters c = (c0, c1, c2, c3) (uint64 holding uint32)."""
    c0, c1, c2, c3 = (np.asarray(v, np.uint64) & M32 for v in c)
    k0, k1 = np.uint64(k0), np.uint64(k1)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ k0) & M32, p1 & M32, ((p0 >> np.uint64(32)) ^ c3 ^ k1) & M32, p0 & M32
        k0 = (k0 + np.uint64(0x9E3779B9)) & M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & M32
    return c0, c1, c2, c3


def host_payload(k0, k1, lo, hi, kp):
    """Payload bits 128 j .. 128 j + 127 from the Philox block (frame, 0xffffffff - j)."""
    pay = np.zeros((lo.size, kp), np.int8)
    for j in range((kp + 127) // 128):
        c2 = np.full(lo.size, 0xFFFFFFFF - j, np.uint64)
        x, y, z, w = philox4x32((lo, hi, c2, np.zeros(lo.size, np.uint64)), k0, k1)
        r0, r1 = (y << np.uint64(32)) | x, (w << np.uint64(32)) | z
        for q in range(128 * j, min(kp, 128 * j + 128)):
            word = r0 if (q & 127) < 64 else r1
            pay[:, q] = ((word >> np.uint64(q & 63)) & np.uint64(1)).astype(np.int8)
    return pay


def host_bm(a, bb):
    """bm_pair (scl_kernels.hip) in numpy float32: the pair of normals of Philox outputs a, bb."""
    u1 = (((a >> np.uint64(11)).astype(np.float64) + 1.0) * 2.0 ** -53).astype(np.float32)
    u2 = (bb >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
    rad = np.sqrt(np.float32(-1.3862943611198906) * np.log2(u1))
    ang = np.float32(2 * np.pi) * u2
    return (rad * np.cos(ang)).astype(np.float64), (rad * np.sin(ang)).astype(np.float64)


def host_stream(seed, stream_id, frame0, B, N, info, K, kp, crc, ebno_db, rate, E=0, order=None):
    k0 = seed & 0xFFFFFFFF
    k1 = ((seed >> 32) ^ ((stream_id * 0x85EBCA6B) & 0xFFFFFFFF)) & 0xFFFFFFFF
    fr = np.arange(frame0, frame0 + B, dtype=np.uint64)
    lo, hi = fr & M32, fr >> np.uint64(32)
    pay = host_payload(k0, k1, lo, hi, kp)
    msg = attach_crc(pay, crc) if crc else pay
    u = np.zeros((B, N), np.int8)
    u[:, info] = msg
    cw = _encode(u)
    Etot = E or N
    nvar = 1.0 / (2.0 * rate * 10 ** (ebno_db / 10.0))
    llr = np.empty((B, Etot))
    for q in range((Etot + 127) // 128):
        c2 = np.arange(64, dtype=np.uint64) + np.uint64(64 * q)
        cx, cy, cz, cw2 = philox4x32((lo[:, None], hi[:, None], c2[None, :], np.zeros((1, 64), np.uint64)), k0, k1)
        a, bb = (cy << np.uint64(32)) | cx, (cw2 << np.uint64(32)) | cz
        zz = host_bm(a, bb)
        for h in range(2):
            p = np.arange(64) + 64 * h + 128 * q
            ok = p < Etot
            pos = order[p[ok] % N] if E else p[ok]
            sym = 1.0 - 2.0 * cw[:, pos]
            llr[:, p[ok]] = (sym + np.sqrt(nvar) * zz[h][:, ok]) * (2.0 / nvar)
    return msg, llr


def _encode(u):
    x = u.copy().astype(np.int8)
    N = x.shape[1]
    st = 1
    while st < N:
        for i in range(N):
            if not (i & st):
                x[:, i] ^= x[:, i + st]
        st <<= 1
    return x


@pytest.mark.parametrize("N,K,crc,E", [(128, 64, "0x1864CFB", 0), (64, 40, "0x1864CFB", 0), (32, 16, None, 0),
                                       (128, 88, "0x1864CFB", 0), (128, 64, "0x1864CFB", 300),
                                       (128, 64, "0x1864CFB", 100), (256, 128, "0x1864CFB", 0),
                                       (512, 300, "0x1864CFB", 0), (1024, 512, None, 0),
                                       (256, 100, "0x1864CFB", 300), (512, 256, "0x1864CFB", 400)])
def test_channel_stream(N, K, crc, E):
    info = construct_info_set(N, K)
    dec = _native.Decoder(N, info, 2, crc)
    deg = dec.crc_deg
    kp = K - deg
    order = None
    if E:
        dec.set_rate_match(E)
        order = _order(N).astype(np.int64)  # symbol p = x[order[p % N]] (interleaver.py:10-23)
    B, frame0, seed, sid = 777, 123456789, 0x1234ABCD5678, 42
    rate = K / (E or N)
    W = dec.W
    with _native.DeviceArena(dec) as mem:
        d_llr = mem.alloc(B * (E or N) * 8)
        d_msg = mem.alloc(B * W * 8)
        dec.channel_device(seed, sid, 3.0, rate, kp, frame0, B, d_llr, d_msg)
        llr = mem.download(d_llr, B * (E or N) * 8, np.float64).reshape(B, E or N)
        words = mem.download(d_msg, B * W * 8, np.uint64).reshape(B, W)
    msg, ref = host_stream(seed, sid, frame0, B, N, info, K, kp, crc, 3.0, rate, E, order)
    got = ((words[:, :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).reshape(B, -1)[:, :K]
    np.testing.assert_array_equal(got.astype(np.int8), msg)
    # normals within 2e-5 (fp32 hardware vs libm transcendentals), i.e. LLRs within 2e-5 * 2 / sigma
    sig = np.sqrt(1.0 / (2.0 * rate * 10 ** 0.3))
    err = np.abs(llr - ref) * sig / 2.0
    assert err.max() < 2e-5 and np.median(err) < 1e-6, (err.max(), np.median(err))


@pytest.mark.parametrize("kp", [40, 200])
def test_uncoded_stream(kp):
    """The uncoded BPSK baseline (run_fer_sweep.py:111-121) counts the errors of the same
    payload bits as the TX chain with its own noise blocks (frame, 0x40000000 + c)."""
    info = construct_info_set(256, kp)
    dec = _native.Decoder(256, info, 2, None)
    B, frame0, seed, sid, ebno = 3000, 77, 0x5EED, 9, 1.0
    nc = _native.PSCL_NCOUNT
    with _native.DeviceArena(dec) as mem:
        d_cnt = mem.alloc(nc * 8)
        mem.memset(d_cnt, 0, nc * 8)
        dec.uncoded_device(seed, sid, ebno, kp, frame0, B, d_cnt)
        cnt = mem.download(d_cnt, nc * 8, np.int64)
    k0 = seed & 0xFFFFFFFF
    k1 = ((seed >> 32) ^ ((sid * 0x85EBCA6B) & 0xFFFFFFFF)) & 0xFFFFFFFF
    fr = np.arange(frame0, frame0 + B, dtype=np.uint64)
    lo, hi = fr & M32, fr >> np.uint64(32)
    pay = host_payload(k0, k1, lo, hi, kp)
    nvar = 1.0 / (2.0 * 10 ** (ebno / 10.0))
    err = np.zeros((B, kp), bool)
    amb = np.zeros((B, kp), bool)
    for c in range((kp + 1) // 2):
        c2 = np.full(B, 0x40000000 + c, np.uint64)
        cx, cy, cz, cw2 = philox4x32((lo, hi, c2, np.zeros(B, np.uint64)), k0, k1)
        a, bb = (cy << np.uint64(32)) | cx, (cw2 << np.uint64(32)) | cz
        zz = host_bm(a, bb)
        for h in range(2):
            q = 2 * c + h
            if q < kp:
                y = (1.0 - 2.0 * pay[:, q]) + np.sqrt(nvar) * zz[h]
                err[:, q] = (y < 0.0) != (pay[:, q] == 1)
                amb[:, q] = np.abs(y) < 1e-4  # decisions the fp32 tolerance could flip
    assert cnt[_native.CNT_FRAMES] == B
    n_amb = int(amb.sum())
    # (|y| < 1e-4 holds for ~3.6e-5 of the decisions at 1 dB: ~22 expected of 6e5 at kp = 200)
    assert n_amb < 60
    assert abs(cnt[_native.CNT_FRAME_ERR] - int(err.any(axis=1).sum())) <= n_amb
    assert abs(cnt[_native.CNT_BIT_ERR] - int(err.sum())) <= n_amb


def test_simulate_uncoded_fused_equals_uncoded_kernel():
    """pscl_simulate counts the uncoded baseline inside the TX launch (N <= 128): the same
    frames' uncoded FER/BER counters as the stand-alone uncoded_device launch, exactly."""
    info = construct_info_set(128, 64)
    dec = _native.Decoder(128, info, 8, "0x1864CFB")
    B, frame0, seed, sid, ebno = 200_000, 1000, 0xABC, 50, 4.0
    nc = _native.PSCL_NCOUNT
    sim = dec.simulate(seed, sid, ebno, 0.5, 40, frame0, B, 0, include_uncoded=True)
    with _native.DeviceArena(dec) as mem:
        d_cnt = mem.alloc(nc * 8)
        mem.memset(d_cnt, 0, nc * 8)
        dec.uncoded_device(seed, sid, ebno, 40, frame0, B, d_cnt)
        unc = mem.download(d_cnt, nc * 8, np.int64)
    np.testing.assert_array_equal(sim[2], unc)
    assert unc[_native.CNT_FRAMES] == B and 0.1 < unc[_native.CNT_FRAME_ERR] / B < 0.5
