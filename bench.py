"""Headline benchmark: decoded frames/s, P(128,64)+CRC-24 SCL L=8 at Eb/N0 = 5 dB (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W --frames B --list L --ebno 5.0]

One step = one pass of the hot path over one batch of B frames per GPU that is already
resident in HBM: SCL decode (fp64, bit-exact to the reference) + CRC selection + FER/BER
counting, i.e. run_fer_sweep.py:79-109 without the TX chain.  The batches are generated
on the device before the timed region by the Philox TX kernel (payload -> CRC-24 ->
polar encode -> BPSK -> AWGN -> LLR), distinct frames per step and per rank.

The line also carries
  parity        the step-0 batch decoded again after the timed region and compared frame by
                frame (best bits, CRC flag, best index) with the oracle's outputs for the
                frames the CPU baseline decoded (oracle/: C restatement of decode_scl);
  roofline      HBM (algorithmic bytes / live launch time) and, from the committed rocprofv3
                PMC entry of the SAME library build (profiles/pmc_traffic.json, keyed by the
                library's source hash), the VALU issue bound priced per instruction class;
  extra_configs BASELINE configs 2 (L=4), 4 (DL-SCL L=4 + 8 flips, beta_M4) and 5 (NR
                E=256 L=8): ms/step, frames/s, FER (z vs the reference's results/fer_M4.csv
                where one applies) and an oracle parity sample each; config 3 (L=8 FER sweep
                4.0-6.5 dB with DL-SCL beta_M8) through run_fer_sweep --rng philox: wall time
                and frames/s per SNR point, FER z at 5 dB.

Multi-GPU: one process per GPU (torchrun), frames sharded by global frame index, no
data-path collective; one RCCL all-reduce of the error counters and one of the timings.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
# OpenMP workers (the oracle's cpu_baseline and parity runs) sleep as soon as a parallel region
# ends: spinning workers -- one per CPU of the affinity mask -- otherwise eat the process's cgroup
# CPU quota and slow the host-bound GPU legs that follow (config 4's launches, the sweep's Python).
# Set before libgomp loads (torch or the oracle), so it applies to both.
os.environ.setdefault("OMP_WAIT_POLICY", "PASSIVE")

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
POLY = "0x1864CFB"
# reference CRC-fail frame errors out of 2000 at 5 dB, seed 0 (results/fer_M{8,4}.csv:2)
REF_ERRS = {("scl", 8): 26, ("dl", 8): 20, ("scl", 4): 91, ("dl", 4): 71}
# multi-rank bounds: the process group's own timeout (a rank that never joins fails the others'
# init and collectives instead of hanging to the library default), and launch_ranks' watchdog --
# no rank finishing a stage for this long ends the job (the first `import torch` on a fresh box
# takes 1-2 minutes; the longest stage, the oracle legs on rank 0, well under one)
PG_TIMEOUT_S = 600
RANK_STALL_S = 480.0

# VALU issue peak of MI355X per instruction class (MI355X_MICROARCH.md, constants table):
# 256 CUs x 4 SIMD-32 at 2.4 GHz; a wave64 instruction takes 2 SIMD cycles (fp32/int/logic,
# moves, DPP, selects, compares: 32 lanes per cycle, with more than one wave per SIMD), 4 for
# fp64 add/mul/fma (16 lanes per cycle), 8 for transcendentals.
SIMDS, CLOCK_HZ = 256 * 4, 2.4e9
CYC_F64, CYC_TRANS, CYC_OTHER = 4, 8, 2


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames", type=int, default=1_000_000, help="frames per GPU per step")
    ap.add_argument("--list", type=int, default=8)
    ap.add_argument("--ebno", type=float, default=5.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=16.0, help="budget for the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--retries", type=int, default=0,
                    help="DL-SCL flip retries per CRC-failing frame (BASELINE config 4: --list 4 --retries 8)")
    ap.add_argument("--beta", type=str, default="auto",
                    help="flip metric .npy ('auto': tests/golden/beta_M{L}.npy, the reference checkpoint; 'none')")
    ap.add_argument("--nr-E", type=int, default=0,
                    help="NR config 5: (128,88) = 64 payload + CRC-24 bits, rate matched to E transmitted "
                         "bits (run_ber_sweep.py nr_polar_scl); the TX kernel interleaves/repeats, the "
                         "decoder de-rate-matches in its channel staging")
    ap.add_argument("--tune", type=str, default="",
                    help="schedule knobs of the bench's decode handle, k=v[,k=v] (pscl_set_tuning: dl_screen, "
                         "dl_chunks, dl_split, side_priority, post_grid, retry_wpg, dl_lane); A/B tools only")
    ap.add_argument("--extra", choices=["auto", "none"], default="auto",
                    help="auto: also time BASELINE configs 2, 4, 5 (extra_configs) after the headline")
    ap.add_argument("--extra-steps", type=int, default=20)
    ap.add_argument("--extra-parity", type=int, default=50_000, help="oracle parity frames per extra config")
    return ap.parse_args()


def frame_bytes(n_in: int, W: int) -> int:
    """Algorithmic HBM bytes per decoded frame: read n_in fp64 LLRs (N, or E rate matched) and
    W reference words, write W best-candidate words and one flag byte."""
    return n_in * 8 + W * 8 + W * 8 + 1


def pmc_entry(workload_key: str, build_hash: str):
    """The committed rocprofv3 PMC entry of the decode kernel for this workload
    (profiles/pmc_traffic.json), only if it was measured on this exact library build."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None, "no profiles/pmc_traffic.json"
    try:
        e = json.loads(p.read_text()).get(workload_key)
    except Exception as ex:  # malformed file: report, do not guess
        return None, f"unreadable profiles/pmc_traffic.json ({ex})"
    if e is None:
        return None, f"no PMC entry for {workload_key}"
    if e.get("build_hash") != build_hash:
        return None, f"PMC entry for {workload_key} is from build {e.get('build_hash')}, timed build is {build_hash}"
    return e, None


def compute_roofline(e: dict, frames: int, launch_ms: float):
    """VALU issue bound of the dominant kernel: SIMD cycles its measured instruction mix needs
    at the guide's per-class rates, over the SIMD cycles available in the live launch time."""
    ipf = float(e["valu_instr_per_frame"])
    mix = e.get("valu_mix_per_frame") or {}
    f64 = sum(float(mix.get(k, 0.0)) for k in ("add_f64", "mul_f64", "fma_f64"))
    trans = float(mix.get("trans_f64", 0.0)) + float(mix.get("trans_f32", 0.0))
    other = ipf - f64 - trans
    need = (CYC_F64 * f64 + CYC_TRANS * trans + CYC_OTHER * other) * frames  # SIMD cycles per launch
    avail = SIMDS * CLOCK_HZ * launch_ms * 1e-3
    return {"bound": "valu-issue", "unit": "SIMD-cycles/launch", "achieved": need, "peak": avail,
            "frac": need / avail, "instr_per_frame": ipf, "fp64_per_frame": f64, "trans_per_frame": trans,
            "other_per_frame": other, "wave_instr_per_s": ipf * frames / (launch_ms * 1e-3),
            "valu_active_frac_pmc": e.get("valu_active_frac"),
            "cycles_per_valu_instr_pmc": e.get("cycles_per_valu_instr"),
            "build_hash": e.get("build_hash"),
            "note": ("instr/frame and class mix: rocprofv3 PMC of this library build (profiles/pmc_traffic.json); "
                     f"price per wave64 instruction: fp64 {CYC_F64}, transcendental {CYC_TRANS}, other {CYC_OTHER} "
                     f"SIMD cycles (MI355X_MICROARCH.md constants table); {SIMDS} SIMDs x {CLOCK_HZ / 1e9:g} GHz")}


def algorithmic_ops(N: int, K: int, L: int, crc_deg: int = 24):
    """SURVEY.md §8(d)'s algorithmic work per frame, in lane operations, as an upper bound (every
    path live at every phase): per path n N/2 f + n N/2 g LLR ops (fp64) and n N/2 partial-sum
    XORs; N metric updates per path (exp + log1p: two transcendentals, one fp64 add); at each of
    the K information phases a bitonic sort of the 2L children (2L/2 * lg(lg+1)/2 compare-exchanges,
    lg = log2 2L; 80 at L = 8), a compare-exchange being a min and a max of fp64 keys; the CRC as
    one K-column XOR per path (crc_deg <= 32 bits: one int op per column)."""
    n = int(round(math.log2(N)))
    llr, xor = L * n * N, L * n * N // 2
    trans, madd = 2 * L * N, L * N
    m = 2 * L
    lg = int(round(math.log2(m)))
    ce = K * (m // 2) * lg * (lg + 1) // 2
    crc = L * K
    return {"fp64": llr + madd + 2 * ce, "trans": trans, "int": xor + crc,
            "detail": {"llr_ops": llr, "psum_xor": xor, "metric_exp_log1p": trans, "metric_add": madd,
                       "sort_compare_exchanges": ce, "crc_xor": crc}}


def compute_algorithmic(N: int, K: int, L: int, frames: int, launch_ms: float):
    """VALU roofline on the ALGORITHMIC op count: §8(d)'s lane operations per
    frame as wave64 instructions at the guide's per-class rates, over the SIMD cycles of the live
    launch time.  Unlike `compute` (the issued instruction mix), a kernel issuing more instructions
    than the algorithm needs cannot raise this fraction."""
    ops = algorithmic_ops(N, K, L)
    cyc = (CYC_F64 * ops["fp64"] + CYC_TRANS * ops["trans"] + CYC_OTHER * ops["int"]) / 64.0
    avail = SIMDS * CLOCK_HZ * launch_ms * 1e-3
    return {"bound": "valu-algorithmic", "unit": "SIMD-cycles/launch", "achieved": cyc * frames, "peak": avail,
            "frac": cyc * frames / avail, "simd_cycles_per_frame": cyc, "lane_ops_per_frame": ops,
            "note": ("SURVEY.md §8(d) op count (upper bound: all L paths live at every phase; exp and log1p one "
                     f"transcendental each), priced per wave64 instruction at fp64 {CYC_F64}, transcendental "
                     f"{CYC_TRANS}, int {CYC_OTHER} SIMD cycles; {SIMDS} SIMDs x {CLOCK_HZ / 1e9:g} GHz")}


def fer_z(errs: int, frames: int, ref_errs: int, ref_frames: int = 2000):
    """Two-proportion z of errs/frames against the reference's ref_errs/ref_frames."""
    p, p0 = errs / max(frames, 1), ref_errs / ref_frames
    pp = (errs + ref_errs) / (frames + ref_frames)
    se = math.sqrt(max(pp * (1 - pp) * (1 / max(frames, 1) + 1 / ref_frames), 1e-30))
    return (p - p0) / se


class Oracle:
    """The checker (oracle/: C restatement of the reference, OpenMP over frames).  Used for the
    CPU baseline and the parity comparisons only, outside every timed region."""

    def __init__(self):
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle

        self.o = oracle

    def run(self, llr, info, L, retries=0, beta=None):
        if retries > 0:
            bits, ok, _ = self.o.dl_batch(llr, info, L, retries, POLY, beta)
            return bits, ok, None
        return self.o.decode_batch(llr, info, L, POLY, want_idx=True)


def host_internal_llrs(llrE: np.ndarray, N: int) -> np.ndarray:
    """NR received LLRs -> the decoder's internal LLRs (decode_rate_matched_scl's front end,
    scl_nr.py:47-48) with the package's host mirrors, for the oracle."""
    from polar_code_amd.nr.polar import derate_match_polar, subblock_deinterleave

    return np.stack([subblock_deinterleave(derate_match_polar(r, N), N) for r in llrE])


def _cpu_quota():
    """The cgroup CPU quota of this process in CPUs (cgroup v2 cpu.max, v1 cfs files), or None."""
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read_text())
        per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def _timed_sample(fn, n0: int, n_max: int, budget_s: float):
    """Calibrate on n0 frames, then repeat a sample sized for the budget until ~80 % of it is
    spent.  Returns (frames done, seconds, distinct frames per pass, first pass's output)."""
    t0 = time.perf_counter()
    fn(n0)
    rate = n0 / max(time.perf_counter() - t0, 1e-6)
    n = int(min(n_max, max(n0, rate * budget_s)))
    done, dt, first = 0, 0.0, None
    t0 = time.perf_counter()
    while dt < budget_s * 0.8 or done == 0:
        out = fn(n)
        first = first if first is not None else out
        done += n
        dt = time.perf_counter() - t0
    return done, dt, n, first


def cpu_baseline(orc: Oracle, llr_host: np.ndarray, info, L: int, budget_s: float, retries: int = 0, beta=None,
                 product_s: float = 6.0):
    """The oracle timed on the host cores on a bounded sample of the step-0 batch, OpenMP over
    frames, at two thread counts: one per CPU of this process's affinity mask (P = the
    host's usable CPUs) and one per CPU of its cgroup CPU quota (rounded up) when that is fewer --
    more threads than the quota only time-slice (a 256-CPU mask on a 16-CPU quota measured 1.9x
    below the 16-thread figure).  `value` is the faster leg, with its `threads_used`; both legs are
    kept in `legs`.  Beside it the product's own host decoder (pscl_decode_cpu,
    csrc/scl_cpu.cpp) at the winning thread count.  Returns the baseline record and the oracle's
    outputs for the first pass of the larger sample (kept for the parity check)."""
    try:
        aff = sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    P_aff = len(aff) if aff else (os.cpu_count() or 1)
    quota = _cpu_quota()
    Ps = [P_aff]
    if quota and int(math.ceil(quota)) < P_aff:
        Ps.append(max(1, int(math.ceil(quota))))
    what = (f"decode_with_retries (SCL L={L} + up to {retries} flips, beta)" if retries > 0
            else f"decode_scl L={L} + CRC select")
    legs, best, keep = [], None, None
    for P in Ps:
        orc.o.set_num_threads(P)
        n0 = min(max(4000, 8 * P), llr_host.shape[0])
        done, dt, n, first = _timed_sample(lambda k: orc.run(llr_host[:k], info, L, retries, beta), n0,
                                           llr_host.shape[0], budget_s / len(Ps))
        leg = {"value": done / dt, "threads_used": orc.o.num_threads(), "per_thread": done / dt / max(orc.o.num_threads(), 1),
               "why": "one per CPU of the affinity mask" if P == P_aff else "one per CPU of the cgroup quota (ceil)",
               "sample": f"{done} frames ({n} distinct), {dt:.1f} s"}
        legs.append(leg)
        if best is None or leg["value"] > best["value"]:
            best = leg
        if keep is None or n > keep[1]:
            keep = (first, n)
    rec = {"value": best["value"], "unit": "frames/s", "cores": best["threads_used"], "kind": "port",
           "threads_used": best["threads_used"], "host_cpu_count": os.cpu_count(),
           "affinity_cpus": len(aff) if aff is not None else None,
           "affinity_mask": _cpu_ranges(aff) if aff is not None else None,
           "cgroup_cpu_quota": quota,
           "per_thread": best["per_thread"],
           "per_quota_cpu": best["value"] / quota if quota else None,
           "legs": legs,
           "sample": f"{best['sample']} of the step-0 batch (same LLRs as the GPU) through oracle/scl_oracle.c "
                     f"(C restatement of {what}), OpenMP over frames, {best['threads_used']} threads ({best['why']}; "
                     f"the faster of {len(legs)} thread count(s), see legs)"}
    P = best["threads_used"]
    if retries == 0:  # the product's own host decoder (no DL-SCL loop on the host path)
        try:
            from polar_code_amd import _native

            n0 = min(max(4000, 8 * P), llr_host.shape[0])
            cdec = _native.CpuDecoder(llr_host.shape[1], info, L, POLY, threads=P)
            pdone, pdt, pn, _ = _timed_sample(
                lambda k: cdec.decode(llr_host[:k], want_metrics=False, want_cands=False, want_info_llrs=False),
                n0, llr_host.shape[0], product_s)
            rec["product_cpu_decoder"] = {
                "value": pdone / pdt, "unit": "frames/s", "threads_used": P, "per_thread": pdone / pdt / P,
                "sample": f"{pdone} frames ({pn} distinct) through pscl_decode_cpu (csrc/scl_cpu.cpp, the "
                          f"product's host decoder, bit-exact), std::thread over frames, {pdt:.1f} s"}
        except Exception as ex:  # reported, never fatal to the GPU line
            rec["product_cpu_decoder"] = {"error": str(ex)}
    return rec, keep[0], keep[1]


def complete_ref(orc: Oracle, host: np.ndarray, ref, info, L: int, retries: int, beta):
    """The oracle's outputs for the whole step-0 batch, so that parity covers every frame: the
    frames the timed sample did not reach are decoded untimed, on one thread per CPU of the cgroup
    quota (more threads than the quota only slow the oracle down)."""
    n = ref[0].shape[0]
    if n >= host.shape[0]:
        return ref
    q = _cpu_quota()
    if q:
        orc.o.set_num_threads(max(1, min(orc.o.num_threads(), int(math.ceil(q)))))
    rest = orc.run(host[n:], info, L, retries, beta)
    return tuple(None if a is None else np.concatenate([a, b]) for a, b in zip(ref, rest))


def _cpu_ranges(cpus):
    """Compact '0-15,32-47' form of a CPU list."""
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def parity(gpu_best_words: np.ndarray, gpu_flags: np.ndarray, ref, K: int, check_idx: bool):
    """Frames whose best bits, CRC flag or (plain decodes) best index differ from the oracle."""
    from polar_code_amd.dlscl.flip import words_to_bits

    bits, ok, idx = ref
    n = bits.shape[0]
    gb = words_to_bits(gpu_best_words[:n], K)
    gpass = (gpu_flags[:n] & 0x80) != 0
    bad = np.any(gb != bits, axis=1) | (gpass != ok)
    if check_idx and idx is not None:
        bad |= (gpu_flags[:n] & 0x3F).astype(np.int32) != idx
    return {"frames": int(n), "mismatches": int(np.count_nonzero(bad)),
            "compared": "best bits, CRC flag" + (", best index" if check_idx else "") + " vs oracle"}


class Ctx:
    def __init__(self, torch, dev, device_index, dist, rank, world):
        self.torch, self.dev, self.device_index = torch, dev, device_index
        self.dist, self.rank, self.world = dist, rank, world

    def max_over_ranks(self, x: float) -> float:
        if not self.dist:
            return x
        red = self.dev if self.dist.get_backend() == "nccl" else "cpu"
        t = self.torch.tensor([x], dtype=self.torch.float64, device=red)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, v):
        if not self.dist:
            return v.cpu().numpy()
        red = self.dev if self.dist.get_backend() == "nccl" else self.torch.device("cpu")
        t = v.to(red)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t.cpu().numpy()

    def barrier(self):
        if self.dist:
            self.dist.barrier()


TUNE: dict = {}  # --tune


def run_workload(ctx: Ctx, *, L: int, E: int, retries: int, beta, B: int, steps: int, warmup: int, ebno: float,
                 seed: int, keep_buffers: bool = False):
    """Generate the batches on the device, run W untimed + K timed steps (barrier and
    synchronize on both sides, max over ranks), then decode the step-0 batch once more
    (untimed) for the parity check.  Returns the measurements."""
    torch, dev = ctx.torch, ctx.dev
    from polar_code_amd import _native
    from polar_code_amd.polar.polar import construct_info_set

    N, K = 128, (88 if E else 64)
    info = construct_info_set(N, K)
    dec = _native.Decoder(N, info, L, POLY, device=ctx.device_index)
    if E:
        dec.set_rate_match(E)
    if TUNE:
        dec.set_tuning(**TUNE)
    n_in = E or N
    stream = torch.cuda.current_stream(dev)
    dec.set_stream(stream.cuda_stream)
    W = dec.W
    kp = K - 24
    rate = kp / E if E else K / N  # run_ber_sweep.py: R = K_payload / E; run_fer_sweep.py: K / N

    # ---- inputs resident in HBM: distinct frames per (rank, step), generated on device
    nbuf = max(1, min(steps, int(48e9 // (B * n_in * 8))))
    llr = [torch.empty((B, n_in), dtype=torch.float64, device=dev) for _ in range(nbuf)]
    msg = [torch.empty((B, W), dtype=torch.int64, device=dev) for _ in range(nbuf)]
    # decodes run pipelined (pscl_set_pipelined: each step's exact re-decode of its deferred frames,
    # or its DL-SCL retry chains, overlap the next steps), so consecutive steps write rotating output
    # buffers: 2 for plain decodes, 4 for DL-SCL steps (the pipeline depth: a step's buffers are free
    # again at the 4th following step, so the chains of up to three steps run behind the baselines);
    # the final join + synchronize covers every pending re-decode and chain
    pipelined = True
    depth = 4 if retries > 0 else 2
    if pipelined:
        dec.set_pipelined(True, depth=depth)
    best_b = [torch.empty((B, W), dtype=torch.int64, device=dev) for _ in range(depth)]
    flags_b = [torch.empty((B,), dtype=torch.uint8, device=dev) for _ in range(depth)]
    calls = [0]
    counters = torch.zeros(8, dtype=torch.int64, device=dev)
    counters_dl = torch.zeros(8, dtype=torch.int64, device=dev)
    snr_idx = int(round(ebno * 10))
    for i in range(nbuf):
        frame0 = (ctx.rank * nbuf + i) * B
        dec.channel_device(seed, snr_idx, ebno, rate, kp, frame0, B, llr[i].data_ptr(), msg[i].data_ptr())
    torch.cuda.synchronize(dev)

    def step(j, count=True):
        c_scl = counters.data_ptr() if count else 0
        ref = msg[j].data_ptr() if count else 0
        best, flags = best_b[calls[0] % depth], flags_b[calls[0] % depth]
        calls[0] += 1
        if retries > 0:  # SCL + DL-SCL retry rounds, all on the device
            dec.dlscl_device(llr[j].data_ptr(), B, retries, beta=beta, d_best=best.data_ptr(),
                             d_flags=flags.data_ptr(), d_ref=ref, k_payload=kp, d_counters_scl=c_scl,
                             d_counters_dl=counters_dl.data_ptr() if count else 0)
        else:
            dec.decode_device(llr[j].data_ptr(), B, d_best=best.data_ptr(), d_flags=flags.data_ptr(), d_ref=ref,
                              k_payload=kp, d_counters=c_scl)

    for i in range(warmup):
        step(i % nbuf)
    dec.join()  # (pipelined: the last warmup call's retry rounds, enqueued and finished here)
    torch.cuda.synchronize(dev)
    counters.zero_()
    counters_dl.zero_()
    dec.timing_enable(True)
    ctx.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i % nbuf)
    dec.join()  # the last step's pending work (pipelined: its retry rounds) inside the timed region
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    ctx.barrier()
    (launches, kern_ms), (side_launches, side_ms) = dec.timing_read_split()
    dec.timing_enable(False)
    elapsed = ctx.max_over_ranks(elapsed)
    c = ctx.sum_over_ranks(counters)
    cdl = ctx.sum_over_ranks(counters_dl)
    # untimed: the step-0 batch once more, outputs kept for the parity check
    step(0, count=False)
    best, flags = best_b[(calls[0] - 1) % depth], flags_b[(calls[0] - 1) % depth]
    dec.sync()
    torch.cuda.synchronize(dev)
    res = {"N": N, "K": K, "W": W, "L": L, "E": E, "B": B, "n_in": n_in, "info": info, "retries": retries,
           "elapsed": elapsed, "launches": launches, "kern_ms": kern_ms, "side_launches": side_launches,
           "side_ms": side_ms, "c": c, "cdl": cdl, "kp": kp,
           "rate": rate, "build_hash": _native.build_hash(), "pipelined": pipelined,
           "best0": best.cpu().numpy().view(np.uint64), "flags0": flags.cpu().numpy()}
    if keep_buffers:
        res["llr0"] = llr[0]
    del llr, msg, best, flags, best_b, flags_b
    dec.close()
    torch.cuda.empty_cache()
    return res


def extra_configs(args, ctx: Ctx, orc: Oracle | None):
    """BASELINE configs 2, 4, 5 (1 GPU each per rank, frame-sharded like the headline)."""
    cfgs = [
        ("config2_scl_L4", dict(L=4, E=0, retries=0), "scl", 4),
        ("config4_dlscl_L4_r8_beta4", dict(L=4, E=0, retries=8), "dl", 4),
        ("config5_nr_E256_L8", dict(L=8, E=256, retries=0), None, None),
    ]
    out = {}
    for name, kw, ref_kind, ref_L in cfgs:
        beta = np.load(ROOT / "tests" / "golden" / "beta_M4.npy") if kw["retries"] else None
        r = run_workload(ctx, **kw, beta=beta, B=args.frames, steps=args.extra_steps, warmup=2, ebno=args.ebno,
                         seed=args.seed, keep_buffers=orc is not None)
        heartbeat(name)
        if ctx.rank != 0:
            continue
        c, cdl = r["c"], r["cdl"]
        frames = int(c[0])
        rec = {"ms_per_step": r["elapsed"] * 1e3 / args.extra_steps,
               "value": args.frames * args.extra_steps * ctx.world / r["elapsed"], "unit": "frames/s",
               "steps": args.extra_steps, "frames_per_gpu_per_step": args.frames,
               "main_stream_kernel_ms_per_step": r["kern_ms"] / args.extra_steps, "main_stream_launches": r["launches"],
               "side_stream_kernel_ms_per_step": r["side_ms"] / args.extra_steps, "side_stream_launches": r["side_launches"],
               "kernel": ("scl_lane_kernel<4> screening + scl128_kernel<4> exact re-decode (pipelined)"
                          if name.startswith("config2") else
                          "scl_lane_kernel<4> baseline + retry rounds beside the next step's baseline: scl_lane_kernel<4,FS>"
                          " screened warm-started retry decodes, scl128_kernel<4,FS> exact decodes of the deferred entries"
                          " (side chain), dl_post_kernel" if name.startswith("config4") else
                          "scl_lane_kernel<8,NR> screening (de-rate-match as the rows are loaded) +"
                          " scl128_kernel<8,CH,CODE=2> exact re-decode (pipelined)"),
               "kernel_timing": ("HIP events around each decode launch: main stream = the screening (plain) or "
                                 "baseline (DL-SCL) decode of each step; side streams = DL-SCL retry decodes, "
                                 "which overlap the main stream (the sums are not additive in wall time)"),
               "roofline": extra_roofline(r, args.extra_steps),
               "fer": {"frames": frames, "frame_errors": int(c[1]), "fer": c[1] / max(frames, 1),
                       "payload_fer": c[3] / max(frames, 1)}}
        if kw["retries"]:
            rec["dl_scl"] = {"frame_errors": int(cdl[1]), "fer": cdl[1] / max(cdl[0], 1),
                             "redecodes_per_frame": cdl[5] / max(cdl[0], 1), "beta": "tests/golden/beta_M4.npy"}
        if ref_kind:
            rec["fer"]["reference"] = f"results/fer_M{ref_L}.csv:2 fer_scl {REF_ERRS[('scl', ref_L)]}/2000"
            rec["fer"]["z_vs_reference"] = fer_z(int(c[1]), frames, REF_ERRS[("scl", ref_L)])
            if kw["retries"]:
                rec["dl_scl"]["reference"] = f"results/fer_M{ref_L}.csv:2 fer_dl {REF_ERRS[('dl', ref_L)]}/2000"
                rec["dl_scl"]["z_vs_reference"] = fer_z(int(cdl[1]), int(cdl[0]), REF_ERRS[("dl", ref_L)])
        if orc is not None:
            n = min(args.extra_parity, args.frames)
            host = r["llr0"][:n].cpu().numpy()
            if kw["E"]:
                host = host_internal_llrs(host, 128)
            ref = orc.run(host, r["info"], kw["L"], kw["retries"], beta)
            rec["parity"] = parity(r["best0"], r["flags0"], ref, r["K"], check_idx=kw["retries"] == 0)
        out[name] = rec
        del r
        ctx.torch.cuda.empty_cache()
    return out


def extra_roofline(r: dict, steps: int) -> dict:
    """Roofline of an extra config's dominant kernel (its main-stream decode: the screening pass of
    a plain decode, the baseline decode of a DL-SCL step): algorithmic HBM bytes per frame x B over
    that kernel's mean live duration, the PMC-priced issue bound where a PMC entry of this build
    and workload exists, and the algorithmic VALU fraction."""
    B, L, N, K = r["B"], r["L"], r["N"], r["K"]
    dom_ms = r["kern_ms"] / max(r["launches"], 1)
    fb = frame_bytes(r["n_in"], r["W"])
    achieved = fb * B / (dom_ms * 1e-3) / 1e9
    wkey = f"scl_L{L}_N{N}_K{K}_B{B}" + (f"_E{r['E']}" if r["E"] else "") + (f"_dl{r['retries']}" if r["retries"] else "")
    e, why = pmc_entry(wkey, r["build_hash"])
    return {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
            "traffic": float(e["hbm_bytes_per_launch"]) if e and "hbm_bytes_per_launch" in e else None,
            "kernel": (dominant_kernel(N, K, L, r["E"], r["retries"])),
            "avg_launch_ms": dom_ms, "bytes_per_frame": fb, "pmc": why or "matched build",
            "compute": compute_roofline(e, B, dom_ms) if e and "valu_instr_per_frame" in e else None,
            "compute_algorithmic": compute_algorithmic(N, K, L, B, dom_ms),
            "step_hbm_gbs": fb * B * steps / r["elapsed"] / 1e9}


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N fresh rank processes (one per GPU, the
    same command line) with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, relay rank 0's output
    and return non-zero if any rank fails.  The parent never imports torch or touches the GPU
    (ranks are children, not exec'd replacements)."""
    import signal
    import subprocess

    import tempfile

    port = free_port()
    hb_dir = tempfile.mkdtemp(prefix="pscl_bench_hb_")
    stall_s = float(os.environ.get("PSCL_RANK_STALL_S", str(RANK_STALL_S)))
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PSCL_BENCH_CHILD="1",
                   PSCL_BENCH_HEARTBEAT=hb_dir)
        procs.append(subprocess.Popen([sys.executable, "-u", str(Path(__file__).resolve()), *sys.argv[1:]],
                                      env=env, stdout=None if r == 0 else subprocess.DEVNULL))
    rcs = [None] * n
    t_launch = time.time()

    def last_progress() -> float:
        """Newest heartbeat of any rank (heartbeat(): one per finished stage), else the launch."""
        t = t_launch
        for f in Path(hb_dir).glob("rank*"):
            try:
                t = max(t, f.stat().st_mtime)
            except OSError:
                pass
        return t

    def stop_all():
        for i, p in enumerate(procs):
            if rcs[i] is None:
                p.send_signal(signal.SIGTERM)
        for i, p in enumerate(procs):
            try:
                rcs[i] = p.wait(timeout=30) if rcs[i] is None else rcs[i]
            except subprocess.TimeoutExpired:
                p.kill()
                rcs[i] = p.wait()

    stalled = False
    try:
        while any(rc is None for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    rcs[i] = p.poll()
            bad = [i for i, rc in enumerate(rcs) if rc not in (None, 0)]
            if bad:  # one rank failed: the others would wait in a collective forever
                stop_all()
                break
            # no rank finished a stage within the bound: a rank that never joined the process group
            # (or hangs in a collective) holds every other one in a collective -- end the job
            if any(rc is None for rc in rcs) and time.time() - last_progress() > stall_s:
                stalled = True
                stop_all()
                break
            time.sleep(0.2)
    except KeyboardInterrupt:
        for p in procs:
            p.kill()
        raise
    finally:
        import shutil

        shutil.rmtree(hb_dir, ignore_errors=True)
    if stalled:
        sys.stderr.write(f"bench.py: no rank progressed for {stall_s:g} s (PSCL_RANK_STALL_S); ranks stopped: "
                         f"{rcs}\n")
        return 1
    failed = [(i, rc) for i, rc in enumerate(rcs) if rc != 0]
    if failed:
        sys.stderr.write(f"bench.py: rank(s) failed: {failed}\n")
        return 1
    return 0


def heartbeat(stage: str) -> None:
    """A rank finished a stage: touch its heartbeat file for launch_ranks' stall watchdog (no-op
    outside bench.py's own launcher)."""
    d = os.environ.get("PSCL_BENCH_HEARTBEAT")
    if d:
        try:
            Path(d, f"rank{os.environ.get('RANK', '0')}").write_text(f"{time.time():.3f} {stage}\n")
        except OSError:
            pass


def dominant_kernel(N, K, L, E, retries):
    """The kernel the step's dominant launch runs (pscl_launch_decode's choice for a plain or
    DL-SCL baseline decode of this configuration)."""
    if N == 128 and L in (4, 8) and ((K == 64 and not E) or (K == 88 and E)):  # (pscl_lane_available)
        return (f"scl_lane_kernel<{L}{'' if K == 64 else ',NR'}> screening pass"
                + (" (DL-SCL baseline)" if retries else ""))
    if N == 128 and L <= 8 and (E or retries):
        return f"scl128_kernel<{L}> " + ("baseline decode" if retries else "screening pass")
    if L in (4, 8, 16, 32) and not E and not retries:  # (any other information set, N = 128..1024)
        return f"scl_lane_long_kernel<N={N},{L}> screening pass"
    return "scl_long_kernel" if N > 128 else "scl_decode_kernel"


def config3_sweep(args, ctx: Ctx):
    """BASELINE config 3 through the product path: run_fer_sweep --rng philox (the whole sweep
    enqueued on a pipelined handle: pscl_simulate_device per block -- TX, uncoded baseline, SCL +
    DL-SCL with beta_M8, counters -- each block's retry chains overlapping the next point's TX and
    baseline), L = 8, 4.0-6.5 dB in 0.5 dB steps, args.frames frames per GPU per point.  Timed as
    one run (max over ranks, Python included), plus a 5 dB-only run for the per-point rate; FER per
    point and the 5 dB z-scores against results/fer_M8.csv."""
    import contextlib
    import io
    import tempfile

    from polar_code_amd.eval import run_fer_sweep as rfs

    frames = args.frames * ctx.world
    beta = str(ROOT / "tests" / "golden" / "beta_M8.npy")

    def run(lo, hi, seed, td):
        a = rfs.build_argparser().parse_args(
            ["--M", "8", "--frames", str(frames), "--snr_lo", f"{lo:g}", "--snr_hi", f"{hi:g}", "--snr_step", "0.5",
             "--retries", "8", "--beta", beta, "--rng", "philox", "--include_uncoded", "--no_plot", "--seed",
             str(seed), "--out_dir", td, "--plot_dir", td])
        ctx.barrier()
        ctx.torch.cuda.synchronize(ctx.dev)
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            rows = rfs.run_sweep(a)
        ctx.torch.cuda.synchronize(ctx.dev)
        return rows, ctx.max_over_ranks(time.perf_counter() - t0)

    with tempfile.TemporaryDirectory() as td:
        # untimed warm-up (handles, device buffers at the timed sizes, beta upload) at another seed
        run(4.0, 4.5, args.seed + 1, td)
        rows, total_t = run(4.0, 6.5, args.seed, td)
        rows5, t5 = run(5.0, 5.0, args.seed, td)
    from polar_code_amd import _native

    _native.release_decoders()  # (the sweep's handle and its streams: the next legs start clean)
    pts = []
    for row in rows:
        pt = {"snr_db": row["snr_db"], "frames": frames, "fer_scl": row["fer_scl"], "fer_dl": row["fer_dl"],
              "fer_uncoded": row["fer_uncoded"], "avg_retries": row["avg_retries"]}
        if abs(row["snr_db"] - 5.0) < 1e-9:
            pt["z_scl_vs_reference"] = fer_z(int(round(row["fer_scl"] * frames)), frames, REF_ERRS[("scl", 8)])
            pt["z_dl_vs_reference"] = fer_z(int(round(row["fer_dl"] * frames)), frames, REF_ERRS[("dl", 8)])
        pts.append(pt)
    return {"workload": "run_fer_sweep --M 8 --retries 8 --beta beta_M8 --rng philox --include_uncoded, "
                        "4.0-6.5 dB step 0.5 (one pipelined pass: pscl_simulate_device per block)",
            "frames_per_point": frames, "wall_s": total_t, "value": frames * len(pts) / total_t,
            "unit": "frames/s (SCL + DL-SCL + uncoded per frame, whole sweep)", "points": pts,
            "kernels": ("channel_kernel TX (+ uncoded count) + scl_lane_kernel<8> baseline + retry rounds: "
                        "scl_lane_kernel<8,FS> screened retry decodes (chains beside the next point's baseline, "
                        "or of >= 24576 entries) or scl128_kernel<8,FS> exact ones, exact re-decodes of the "
                        "deferred entries, dl_post_kernel"),
            "point_5db": {"wall_s": t5, "frames_per_s": frames / t5, "fer_scl": rows5[0]["fer_scl"],
                          "fer_dl": rows5[0]["fer_dl"]},
            "reference": "results/fer_M8.csv:2 (5 dB): fer_scl 26/2000, fer_dl 20/2000"}


def main():
    args = parse()
    if args.tune:
        TUNE.update({k: int(v) for k, v in (kv.split("=") for kv in args.tune.split(","))})
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (one rank per GPU)")
    if os.environ.get("PSCL_BENCH_STALL_RANK") == str(rank):  # (test hook: a rank that never joins)
        time.sleep(1e6)
    import datetime

    import torch

    # PSCL_BENCH_DIST_ONLY=1 (launcher tests on CPU): the process group and one barrier, no GPU
    dist_only = os.environ.get("PSCL_BENCH_DIST_ONLY") == "1"
    dev, device_index = None, 0
    if not dist_only:
        # one process per GPU; PSCL_SHARE_GPU=1 lets a rehearsal put several ranks on fewer GPUs
        ndev = torch.cuda.device_count()
        device_index = local % ndev if os.environ.get("PSCL_SHARE_GPU") == "1" else local
        torch.cuda.set_device(device_index)
        dev = torch.device("cuda", device_index)
    dist = None
    # a process group under any launcher, world 1 included (the RCCL collectives then run on one
    # GPU exactly as on eight); none for a plain `python bench.py`
    if world > 1 or ("MASTER_ADDR" in os.environ and "WORLD_SIZE" in os.environ):
        import torch.distributed as dist

        backend = os.environ.get("PSCL_DIST_BACKEND", "gloo" if dist_only else "nccl")  # nccl == RCCL over xGMI
        timeout = datetime.timedelta(seconds=float(os.environ.get("PSCL_PG_TIMEOUT_S", str(PG_TIMEOUT_S))))
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=dev, timeout=timeout)
        else:
            dist.init_process_group(backend=backend, timeout=timeout)
        heartbeat("process group")
    if dist_only:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    ctx = Ctx(torch, dev, device_index, dist, rank, world)

    E, L, B = args.nr_E, args.list, args.frames
    beta = None
    if args.retries > 0 and args.beta != "none":
        bp = ROOT / "tests" / "golden" / f"beta_M{L}.npy" if args.beta == "auto" else Path(args.beta)
        beta = np.load(bp) if bp.exists() else None
    r = run_workload(ctx, L=L, E=E, retries=args.retries, beta=beta, B=B, steps=args.steps, warmup=args.warmup,
                     ebno=args.ebno, seed=args.seed, keep_buffers=(rank == 0))
    heartbeat("headline")
    N, K, W, n_in, info, kp = r["N"], r["K"], r["W"], r["n_in"], r["info"], r["kp"]
    c, cdl, elapsed = r["c"], r["cdl"], r["elapsed"]
    frames_total = B * args.steps * world

    cpu = par = None
    orc = Oracle() if (rank == 0 and not args.no_cpu_baseline) else None
    host = None
    if orc is not None:
        host = r["llr0"][: min(B, 1_000_000)].cpu().numpy()
        if E:
            host = host_internal_llrs(host[: min(host.shape[0], 100_000)], N)
    r.pop("llr0", None)
    torch.cuda.empty_cache()
    extra = None
    if args.extra == "auto" and not E and args.retries == 0 and L == 8:
        # (the sweep first: the extra configs' oracle parity checks run the oracle on every CPU of
        # the affinity mask, after which the host-timed sweep measured ~4 % slower)
        sweep = config3_sweep(args, ctx)
        heartbeat("config3 sweep")
        extra = extra_configs(args, ctx, orc)
        heartbeat("extra configs")
        if rank == 0:
            extra["config3_sweep_L8"] = sweep
    # the CPU legs after every timed GPU leg: the oracle's workers (one per CPU of the affinity mask,
    # on a cgroup quota of fewer CPUs) measured to slow the host-bound legs that followed them (the
    # config-3 sweep 281 -> 271 M frames/s, its 5 dB point 4.54 -> 4.72 ms)
    if orc is not None:
        if world == 1:
            cpu, ref, n = cpu_baseline(orc, host, info, L, args.cpu_seconds, args.retries, beta)
            ref = complete_ref(orc, host, ref, info, L, args.retries, beta)
        else:  # the CPU baseline is an N = 1 figure; the step-0 parity check stays (untimed)
            ref = orc.run(host, info, L, args.retries, beta)
        par = parity(r["best0"], r["flags0"], ref, K, check_idx=args.retries == 0)
        host = None
        heartbeat("cpu baseline + parity")

    if rank == 0:
        launches, kern_ms = r["launches"], r["kern_ms"]
        avg_ms = kern_ms / max(launches, 1)
        fb = frame_bytes(n_in, W)
        # main-stream launches: one per step (the screening pass of a plain decode, the baseline
        # decode of a DL-SCL step; the retry decodes run on side streams)
        per_batch_ms = kern_ms / args.steps if args.retries > 0 else avg_ms
        achieved = fb * B / (per_batch_ms * 1e-3) / 1e9
        wkey = f"scl_L{L}_N{N}_K{K}_B{B}" + (f"_E{E}" if E else "") + (f"_dl{args.retries}" if args.retries > 0 else "")
        e, why = pmc_entry(wkey, r["build_hash"])
        traffic = float(e["hbm_bytes_per_launch"]) if e and "hbm_bytes_per_launch" in e else None
        compute = compute_roofline(e, B, per_batch_ms) if e and "valu_instr_per_frame" in e else None
        fer = c[1] / max(c[0], 1)
        ref_scl = REF_ERRS.get(("scl", L)) if not E else None
        dl = None
        if args.retries > 0:
            ref_dl = REF_ERRS.get(("dl", L)) if not E else None
            dl = {"retries": args.retries, "beta": None if beta is None else "tests/golden/beta_M%d.npy" % L,
                  "frame_errors": int(cdl[1]), "fer": cdl[1] / max(cdl[0], 1), "ber": cdl[2] / max(cdl[0] * K, 1),
                  "redecodes": int(cdl[5]), "redecodes_per_frame": cdl[5] / max(cdl[0], 1),
                  "z_vs_reference": fer_z(int(cdl[1]), int(cdl[0]), ref_dl) if ref_dl and args.ebno == 5.0 else None}
        metric = "decoded frames/sec, P(128,64)+CRC24 SCL L=8 @ Eb/N0=5 dB; FER match"
        workload = (f"SCL L={L} P({N},{K})+CRC24 (0x1864CFB) @ Eb/N0={args.ebno:g} dB, "
                    f"{B} frames/GPU/step, decode+CRC select+FER/BER count")
        if E:
            metric = f"decoded frames/sec, NR polar N=128 E={E} K=64+CRC24 SCL L={L}"
            workload = (f"NR SCL L={L} (128,88) rate matched E={E}, R={r['rate']:g} @ Eb/N0={args.ebno:g} dB, {B} "
                        f"frames/GPU/step, de-rate-match + decode + CRC select + FER/BER count")
        if args.retries > 0:
            metric = f"decoded frames/sec, P(128,{K})+CRC24 DL-SCL L={L} + {args.retries} flip retries"
            workload = (f"DL-SCL L={L} + {args.retries} flips (beta) P({N},{K})+CRC24 @ Eb/N0={args.ebno:g} dB, "
                        f"{B} frames/GPU/step, SCL + retry rounds + FER/BER count")
        line = {
            "metric": metric,
            "value": frames_total / elapsed,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: on-device Philox4x32 BPSK/AWGN frames (payload->CRC24->polar->LLR), resident in HBM",
            "config": {"workload": workload, "retries": args.retries, "E": E or None, **({"tuning": TUNE} if TUNE else {}),
                       "N": N, "K": K, "list_size": L, "ebno_db": args.ebno, "frames_per_gpu_per_step": B,
                       "global_batch": B * world, "parallelism": f"frame-sharded x{world}",
                       "collective": dist.get_backend() if dist else None},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS,
                         "traffic": traffic,
                         "kernel": dominant_kernel(N, K, L, E, args.retries),
                         "timed": ("screening launch (pipelined: each step's exact re-decode of its deferred "
                                   "frames overlaps the next step's screening)" if r["pipelined"] else
                                   "decode launches of a step"),
                         "avg_launch_ms": avg_ms, "launches": launches,
                         "main_stream_kernel_ms_per_step": kern_ms / args.steps,
                         "side_stream_kernel_ms_per_step": r["side_ms"] / args.steps,
                         "bytes_per_frame": fb, "build_hash": r["build_hash"], "pmc": why or "matched build",
                         "compute": compute,
                         "compute_algorithmic": compute_algorithmic(N, K, L, B, per_batch_ms)},
            "cpu_baseline": cpu,
            "parity": par,
            "fer": {"frames": int(c[0]), "frame_errors": int(c[1]), "fer": fer, "ber": c[2] / max(c[0] * K, 1),
                    "payload_fer": c[3] / max(c[0], 1), "payload_ber": c[4] / max(c[0] * kp, 1),
                    "reference_fer": ref_scl / 2000 if ref_scl else None,
                    "z_vs_reference": fer_z(int(c[1]), int(c[0]), ref_scl) if ref_scl and args.ebno == 5.0 else None},
            "dl_scl": dl,
            "extra_configs": extra,
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
