"""Generate golden vectors by running the reference implementation (survey container only).

    PYTHONPATH=/root/reference python tests/golden/make_golden.py

Imports heimrih/polar_code's dl_scl_polar package from /root/reference and records its
outputs on seeded inputs as .npz fixtures (inputs + expected outputs only).  The GPU box
never sees the reference: tests read only the committed .npz files.

Fixture sets:
  G1  info sets                         construct_info_set        polar.py:85-103
  G2  CRC attach/check                  attach_crc / check_crc    crc.py:19-56
  G3  polar encode                      encode / _polar_transform polar.py:17-29,106-119
  G4  decode_scl outputs M in {1,2,4,8} x Eb/N0 in {1,3,5,7} dB  scl.py:108-209
  G5  exact-tie cases (noiseless +-50, +-1e6 LLRs)
  G6  decode_scl with force_info_bits (prefix + flip)              scl.py:127-158
  G7  decode_with_retries (beta_M4 and beta=None)                  dlscl/flip.py:65-141
  G8  NR de-rate-match / de-interleave / decode_rate_matched_scl   nr/polar/*
  G9  sc_decode                                                    polar.py:130-168
  G10 odd shapes: N in {2,4,8,16,32,64}, M in {3,5,16}, K=88, no-CRC
  G11 run_ber_sweep rows                                           eval/run_ber_sweep.py
  G12 make_dataset shards (abs_l0, flip_idx, meta)                 train/make_dataset.py:24-121
  G13 train_beta on the G12 shard (CPU, one thread): beta + log      train/train_beta.py:64-161
  G14 longer codes: decode_scl at N in {256, 512, 1024} (incl. forced bits) and sc_decode at N=256
  G15 decode_with_retries on quantised LLRs (exact |L0| / q ties in the flip ranking)  flip.py:104-108
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
if str(REF) not in sys.path:
    sys.path.insert(0, str(REF))

from dl_scl_polar.polar.polar import construct_info_set, encode, sc_decode, _polar_transform  # noqa: E402
from dl_scl_polar.polar.crc import attach_crc, check_crc  # noqa: E402
from dl_scl_polar.polar.scl import decode_scl  # noqa: E402
from dl_scl_polar.dlscl.flip import decode_with_retries  # noqa: E402
from dl_scl_polar.nr.polar import (  # noqa: E402
    derate_match_polar,
    subblock_deinterleave,
    subblock_interleave,
    rate_match_polar,
    decode_rate_matched_scl,
    encode_rate_matched,
)

OUT = Path(__file__).resolve().parent
POLY = "0x1864CFB"


def llr_awgn(rng, code, ebno_db, rate):
    ebno = 10 ** (ebno_db / 10.0)
    nv = 1.0 / (2.0 * rate * ebno)
    noise = rng.normal(0.0, np.sqrt(nv), size=code.size)
    return 2.0 * ((1.0 - 2.0 * code) + noise) / nv


def pack_decode(res, M, K):
    n = len(res["candidates"])
    cands = np.zeros((M, K), np.int8)
    mets = np.full(M, np.nan)
    illr = np.full((M, K), np.nan)
    for i in range(n):
        cands[i] = res["candidates"][i]
        mets[i] = res["metrics"][i]
        illr[i, : len(res["info_llrs"][i])] = res["info_llrs"][i]
    best = -1
    if res["best_path_bits"] is not None:
        for i in range(n):
            if np.array_equal(res["candidates"][i], res["best_path_bits"]):
                best = i
                break
    return n, cands, mets, illr, best


def g1():
    d = {}
    for (N, K) in [(128, 64), (128, 88), (16, 12), (64, 32), (32, 16), (256, 128), (8, 4)]:
        d[f"info_{N}_{K}"] = construct_info_set(N, K)
    np.savez_compressed(OUT / "g1_info_sets.npz", **d)


def g2():
    rng = np.random.default_rng(2)
    pay = rng.integers(0, 2, size=(256, 40), dtype=np.int8)
    att = np.stack([attach_crc(p, POLY) for p in pay])
    cor = att.copy()
    flip = rng.integers(0, 64, size=256)
    cor[np.arange(256), flip] ^= 1
    chk_ok = np.array([check_crc(a, POLY) for a in att])
    chk_bad = np.array([check_crc(c, POLY) for c in cor])
    pay8 = rng.integers(0, 2, size=(64, 8), dtype=np.int8)
    att8 = np.stack([attach_crc(p, "0x17") for p in pay8])
    rnd = rng.integers(0, 2, size=(256, 64), dtype=np.int8)
    chk_rnd = np.array([check_crc(r, POLY) for r in rnd])
    np.savez_compressed(OUT / "g2_crc.npz", payload=pay, attached=att, corrupted=cor, check_ok=chk_ok,
                        check_bad=chk_bad, payload8=pay8, attached8_0x17=att8, random64=rnd, check_random=chk_rnd)


def g3():
    rng = np.random.default_rng(3)
    msg = rng.integers(0, 2, size=(256, 64), dtype=np.int8)
    code = np.stack([encode(m) for m in msg])
    u = rng.integers(0, 2, size=(64, 128), dtype=np.int8)
    xu = np.stack([_polar_transform(v) for v in u])
    np.savez_compressed(OUT / "g3_encode.npz", msg=msg, code=code, u=u, transform=xu)


def decode_set(name, N, K, Ms, snrs, frames, seed, crc=POLY, force_fn=None, extra=None):
    info = construct_info_set(N, K)
    rng = np.random.default_rng(seed)
    d = {"info": info, "N": N, "K": K}
    kp = K - (len(bin(int(crc, 16))) - 3 if crc else 0)
    for M in Ms:
        for snr in snrs:
            llrs, ns, cs, ms, ils, bs, fs = [], [], [], [], [], [], []
            for _ in range(frames):
                pay = rng.integers(0, 2, size=kp, dtype=np.int8)
                msg = attach_crc(pay, crc) if crc else pay
                u = np.zeros(N, np.int8)
                u[info] = msg
                code = _polar_transform(u)
                llr = llr_awgn(rng, code, snr, K / N)
                force = force_fn(rng, K) if force_fn else None
                res = decode_scl(llr, info, M, crc=crc, force_info_bits=force)
                n, c, m, il, b = pack_decode(res, M, K)
                llrs.append(llr)
                ns.append(n)
                cs.append(c)
                ms.append(m)
                ils.append(il)
                bs.append(b)
                fs.append(force if force is not None else np.full(K, -1, np.int8))
            key = f"M{M}_snr{snr:g}"
            d[key + "_llr"] = np.stack(llrs)
            d[key + "_npaths"] = np.array(ns, np.int32)
            d[key + "_cands"] = np.stack(cs)
            d[key + "_metrics"] = np.stack(ms)
            d[key + "_info_llrs"] = np.stack(ils)
            d[key + "_best"] = np.array(bs, np.int32)
            d[key + "_force"] = np.stack(fs)
    d["keys"] = np.array([f"M{M}_snr{s:g}" for M in Ms for s in snrs])
    d["crc"] = np.array(crc if crc else "")
    if extra:
        d.update(extra)
    np.savez_compressed(OUT / f"{name}.npz", **d)


def g5():
    """Exact metric ties: noiseless +-50 and +-1e6 LLRs (survey hard part 1)."""
    info = construct_info_set(128, 64)
    rng = np.random.default_rng(5)
    d = {"info": info}
    for amp in (50.0, 1e6, 3.0):
        for M in (4, 8):
            llrs, ns, cs, ms, ils, bs = [], [], [], [], [], []
            for _ in range(6):
                msg = attach_crc(rng.integers(0, 2, size=40, dtype=np.int8), POLY)
                code = encode(msg)
                llr = np.where(code == 0, amp, -amp).astype(float)
                res = decode_scl(llr, info, M, crc=POLY)
                n, c, m, il, b = pack_decode(res, M, 64)
                llrs.append(llr), ns.append(n), cs.append(c), ms.append(m), ils.append(il), bs.append(b)
            key = f"amp{amp:g}_M{M}"
            d[key + "_llr"] = np.stack(llrs)
            d[key + "_npaths"] = np.array(ns, np.int32)
            d[key + "_cands"] = np.stack(cs)
            d[key + "_metrics"] = np.stack(ms)
            d[key + "_info_llrs"] = np.stack(ils)
            d[key + "_best"] = np.array(bs, np.int32)
    d["keys"] = np.array([f"amp{a:g}_M{M}" for a in (50.0, 1e6, 3.0) for M in (4, 8)])
    np.savez_compressed(OUT / "g5_ties.npz", **d)


def force_prefix_flip(rng, K):
    i = int(rng.integers(0, K))
    f = np.full(K, -1, np.int8)
    f[:i] = rng.integers(0, 2, size=i)
    f[i] = int(rng.integers(0, 2))
    return f


def g7():
    info = construct_info_set(128, 64)
    beta4 = np.load(REF / "checkpoints" / "beta_M4.npy")
    rng = np.random.default_rng(7)
    frames = []
    # collect baseline-failing frames at 2.5 dB, M=4
    while len(frames) < 40:
        msg = attach_crc(rng.integers(0, 2, size=40, dtype=np.int8), POLY)
        llr = llr_awgn(rng, encode(msg), 2.5, 0.5)
        base = decode_scl(llr, info, 4, crc=POLY)
        if not check_crc(base["best_path_bits"], POLY):
            frames.append((llr, msg))
    d = {"info": info, "beta": beta4, "llr": np.stack([f[0] for f in frames]), "msg": np.stack([f[1] for f in frames])}
    for tag, beta in (("beta", beta4), ("none", None)):
        bits, succ, att, tried = [], [], [], []
        for llr, _ in frames:
            r = decode_with_retries(llr, info, 4, 8, crc=POLY, beta=beta)
            bits.append(r["best_path_bits"])
            succ.append(r["success"])
            att.append(len(r["attempts"]))
            t = np.full(8, -1, np.int32)
            t[: len(r["tried_indices"])] = r["tried_indices"]
            tried.append(t)
        d[f"{tag}_bits"] = np.stack(bits)
        d[f"{tag}_success"] = np.array(succ)
        d[f"{tag}_attempts"] = np.array(att, np.int32)
        d[f"{tag}_tried"] = np.stack(tried)
    np.savez_compressed(OUT / "g7_flip.npz", **d)


def g8():
    N, E, Kp, Kc = 128, 256, 64, 24
    info = construct_info_set(N, Kp + Kc)
    rng = np.random.default_rng(8)
    llrE, internal, bits, crcp, pays = [], [], [], [], []
    for _ in range(12):
        pay = rng.integers(0, 2, size=Kp, dtype=np.int8)
        tx = encode_rate_matched(pay, POLY, N, E, info)
        nv = 1.0 / (2.0 * (10 ** 0.2) * Kp / E)
        llr = 2.0 * ((1.0 - 2.0 * tx) + rng.normal(0.0, np.sqrt(nv), size=E)) / nv
        inter = subblock_deinterleave(derate_match_polar(llr, N), N)
        r = decode_rate_matched_scl(llr, POLY, N, E, info, 8)
        llrE.append(llr), internal.append(inter), bits.append(r["best_path_bits"]), crcp.append(r["crc_pass"])
        pays.append(pay)
    x = rng.integers(0, 2, size=N, dtype=np.int8)
    d = dict(info=info, llrE=np.stack(llrE), internal=np.stack(internal), bits=np.stack(bits),
             crc_pass=np.array(crcp), payload=np.stack(pays), ilv_in=x, ilv_out=subblock_interleave(x),
             rm_in=x, rm_out_E200=rate_match_polar(x, 200), rm_out_E100=rate_match_polar(x, 100),
             derate_in=np.linspace(-3, 3, 200), derate_out=derate_match_polar(np.linspace(-3, 3, 200), N),
             derate_in_short=np.linspace(-3, 3, 100), derate_out_short=derate_match_polar(np.linspace(-3, 3, 100), N))
    np.savez_compressed(OUT / "g8_nr.npz", **d)


def g9():
    info = construct_info_set(128, 64)
    rng = np.random.default_rng(9)
    llr = np.stack([llr_awgn(rng, encode(rng.integers(0, 2, 64, dtype=np.int8)), s, 0.5)
                    for s in (0.0, 2.0, 4.0, 6.0) for _ in range(16)])
    # include exact zeros and tiny negatives (SC decides llr < 0)
    llr[0, :8] = 0.0
    llr[1, :8] = -1e-300
    out = np.stack([sc_decode(l, info) for l in llr])
    np.savez_compressed(OUT / "g9_sc.npz", info=info, llr=llr, bits=out)


BER_CONFIGS = {
    "ber_polar_small": ["--scheme", "polar_scl", "--K_payload", "8", "--K_crc", "4", "--E", "16", "--crc_poly", "0x17",
                        "--M", "2", "--EbN0_lo", "6.0", "--EbN0_hi", "6.0", "--EbN0_step", "0.5", "--bits_cap", "64",
                        "--err_cap", "2"],
    "ber_polar_128": ["--scheme", "polar_scl", "--K_payload", "40", "--K_crc", "24", "--E", "128", "--M", "4",
                      "--EbN0_lo", "6.0", "--EbN0_hi", "7.0", "--EbN0_step", "0.5", "--bits_cap", "24000",
                      "--err_cap", "100", "--seed", "3"],
    "ber_dl_128": ["--scheme", "dl_scl", "--K_payload", "40", "--K_crc", "24", "--E", "128", "--M", "4",
                   "--retries", "8", "--beta", "BETA4", "--EbN0_lo", "6.0", "--EbN0_hi", "6.0", "--bits_cap", "8000",
                   "--err_cap", "60", "--seed", "4"],
    "ber_nr_256": ["--scheme", "nr_polar_scl", "--K_payload", "64", "--K_crc", "24", "--E", "256", "--N", "128",
                   "--M", "8", "--EbN0_lo", "4.0", "--EbN0_hi", "4.5", "--EbN0_step", "0.5", "--bits_cap", "9600",
                   "--err_cap", "100", "--seed", "5"],
    "ber_nr_small": ["--scheme", "nr_polar_scl", "--K_payload", "8", "--K_crc", "4", "--E", "16", "--N", "16",
                     "--M", "2", "--EbN0_lo", "5.0", "--EbN0_hi", "5.0", "--bits_cap", "64", "--err_cap", "2",
                     "--crc_poly", "0x17"],
}


def g11():
    """run_ber_sweep rows (CSV text) for several configurations (stop rule, shared stream)."""
    from dl_scl_polar.eval import run_ber_sweep as rb
    import tempfile

    d = {}
    for name, argv in BER_CONFIGS.items():
        argv = [str(REF / "checkpoints" / "beta_M4.npy") if a == "BETA4" else a for a in argv]
        with tempfile.TemporaryDirectory() as td:
            out = Path(td) / "x.csv"
            rows = rb.run(rb.parse_args(argv + ["--out", str(out)]))
            rb.write_csv(rows, out)
            d[name] = np.array(out.read_text())
        d[name + "_argv"] = np.array(" ".join(BER_CONFIGS[name]))
    np.savez_compressed(OUT / "g11_ber.npz", **d)


DATASET_CONFIGS = {"m4_2p5db": ["--M", "4", "--snr_db", "2.5", "--frames", "300", "--seed", "0"],
                   "m8_3db": ["--M", "8", "--snr_db", "3.0", "--frames", "200", "--seed", "1"]}


def g12():
    """make_dataset shards: the reference's generate_samples on small low-SNR runs."""
    from dl_scl_polar.train import make_dataset as md
    import tempfile

    d = {}
    for name, argv in DATASET_CONFIGS.items():
        with tempfile.TemporaryDirectory() as td:
            md.generate_samples(md.build_argparser().parse_args(argv + ["--out", str(Path(td) / "ds")]))
            z = np.load(Path(td) / "ds_part0.npz")
            d[name + "_abs_l0"] = z["abs_l0"]
            d[name + "_flip_idx"] = z["flip_idx"]
            d[name + "_meta"] = np.array(str(z["meta"]))
        d[name + "_argv"] = np.array(" ".join(argv))
    np.savez_compressed(OUT / "g12_dataset.npz", **d)


def g13():
    """train_beta (CPU, 1 thread) on the g12 m4 shard: checkpoint beta and the epoch log."""
    import tempfile
    import torch
    from dl_scl_polar.train import train_beta as tb

    torch.set_num_threads(1)
    z = np.load(OUT / "g12_dataset.npz")
    d = {}
    with tempfile.TemporaryDirectory() as td:
        shard = Path(td) / "ds_part0.npz"
        np.savez_compressed(shard, abs_l0=z["m4_2p5db_abs_l0"], flip_idx=z["m4_2p5db_flip_idx"],
                            meta=z["m4_2p5db_meta"])
        argv = ["--M", "4", "--data", str(shard), "--epochs", "3", "--batch", "16", "--lr", "1e-3",
                "--lambda_l2", "0.25", "--seed", "7", "--val_frac", "0.25", "--cpu"]
        tb.train_beta(tb.build_argparser().parse_args(argv + ["--checkpoint_dir", td, "--log_dir", td]))
        d["beta"] = np.load(Path(td) / "beta_M4.npy")
        d["log"] = np.array((Path(td) / "train_M4.csv").read_text())
        d["argv"] = np.array(" ".join(argv))
    np.savez_compressed(OUT / "g13_train_beta.npz", **d)


def g14():
    """Code lengths above 128 (decode_scl accepts any power of two, scl.py:25-30)."""
    decode_set("g14_n256", 256, 128, [1, 4, 8], [2.0], 6, seed=140)
    decode_set("g14_n256_forced", 256, 128, [4], [2.5], 4, seed=141, force_fn=force_prefix_flip)
    decode_set("g14_n512", 512, 256, [2, 8], [2.0], 3, seed=142)
    decode_set("g14_n1024", 1024, 512, [4], [2.0], 2, seed=143)
    info = construct_info_set(256, 128)
    rng = np.random.default_rng(144)
    llr = np.stack([rng.normal(1.0, 2.0, 256) for _ in range(8)])
    bits = np.stack([sc_decode(x, info) for x in llr])
    np.savez_compressed(OUT / "g14_sc256.npz", info=info, llr=llr, bits=bits)


def g15():
    """Flip-ranking ties: LLRs quantised to a few levels make many decision LLRs |L0| equal
    (min-sum picks the same channel magnitudes), so np.argsort's order among equal keys
    decides the flip.  Also records which SIMD argsort this host's NumPy used."""
    info = construct_info_set(128, 64)
    beta4 = np.load(REF / "checkpoints" / "beta_M4.npy")
    rng = np.random.default_rng(15)
    frames = []
    while len(frames) < 48:
        msg = attach_crc(rng.integers(0, 2, size=40, dtype=np.int8), POLY)
        llr = llr_awgn(rng, encode(msg), 3.0, 0.5)
        llr = np.clip(np.round(llr / 3.0), -3, 3) * 3.0  # levels -9 .. 9, step 3
        base = decode_scl(llr, info, 4, crc=POLY)
        if not check_crc(base["best_path_bits"], POLY):
            frames.append(llr)
    simd = np.__config__.CONFIG["SIMD Extensions"]["found"] if hasattr(np, "__config__") else []
    d = {"info": info, "beta": beta4, "llr": np.stack(frames), "numpy_simd": np.array(" ".join(map(str, simd))),
         "numpy_version": np.array(np.__version__)}
    for tag, beta in (("beta", beta4), ("none", None)):
        bits, succ, att, tried = [], [], [], []
        for llr in frames:
            r = decode_with_retries(llr, info, 4, 8, crc=POLY, beta=beta)
            bits.append(r["best_path_bits"])
            succ.append(r["success"])
            att.append(len(r["attempts"]))
            t = np.full(8, -1, np.int32)
            t[: len(r["tried_indices"])] = r["tried_indices"]
            tried.append(t)
        d[f"{tag}_bits"] = np.stack(bits)
        d[f"{tag}_success"] = np.array(succ)
        d[f"{tag}_attempts"] = np.array(att, np.int32)
        d[f"{tag}_tried"] = np.stack(tried)
    np.savez_compressed(OUT / "g15_dl_ties.npz", **d)


def main():
    if len(sys.argv) > 1:
        for name in sys.argv[1:]:
            globals()[name]()
        return
    g1()
    g2()
    g3()
    decode_set("g4_decode", 128, 64, [1, 2, 4, 8], [1.0, 3.0, 5.0, 7.0], 20, seed=4)
    g5()
    decode_set("g6_forced", 128, 64, [2, 4, 8], [2.0, 5.0], 12, seed=6, force_fn=force_prefix_flip)
    g7()
    g8()
    g9()
    decode_set("g10_n16", 16, 12, [1, 2, 3, 4], [2.0, 6.0], 12, seed=10, crc="0x17")
    decode_set("g10_n32", 32, 20, [2, 5], [3.0], 12, seed=11, crc="0x17")
    decode_set("g10_n64_nocrc", 64, 32, [1, 4], [3.0], 12, seed=12, crc=None)
    decode_set("g10_k88", 128, 88, [8], [3.0], 12, seed=13)
    decode_set("g10_m16", 128, 64, [16], [2.0], 6, seed=14)
    decode_set("g10_n8", 8, 6, [2, 4], [2.0], 12, seed=15, crc="0x5")
    decode_set("g10_n4", 4, 3, [1, 2, 3], [1.0], 12, seed=16, crc=None)
    decode_set("g10_n2", 2, 1, [1, 2], [0.0], 12, seed=17, crc=None)
    g11()
    g12()
    g13()
    g14()
    g15()
    for p in sorted(OUT.glob("*.npz")):
        print(p.name, p.stat().st_size)


if __name__ == "__main__":
    main()
