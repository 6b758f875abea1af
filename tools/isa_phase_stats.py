"""Static per-phase instruction mix of a fully unrolled scl128 kernel (CPU-side analysis).

    hipcc ... -DPSCL_PHASE_MARKERS --cuda-device-only -S scl128_spec.hip -o k.s
    python tools/isa_phase_stats.py k.s <kernel-substring> [info-mask-hex-lo info-mask-hex-hi]

Splits the kernel body at the '; PHASE t' markers (scl128_impl.h) and counts instructions per
class in each phase segment; with the information set it totals by phase kind (frozen/info,
recompute phases t == 0).  The code is straight-line, so static counts approximate the
dynamic mix of the common path (rare wave branches excluded by the reader)."""
import collections
import re
import sys


def klass(op, line):
    if op.startswith("s_"):
        return "salu/ctl"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if "_dpp" in op or "row_" in line or "quad_perm" in line:
        return "dpp"
    for k in ("add_f64", "fma_f64", "mul_f64", "min_f64", "max_f64", "ldexp_f64", "fmac_f64"):
        if k in op:
            return "f64:" + k
    if op.startswith(("v_exp_f32", "v_rcp_f32", "v_log_f32")):
        return "trans"
    if "cndmask" in op:
        return "cndmask"
    if op.startswith("v_cmp"):
        return "cmp"
    if op.startswith(("v_mov", "v_readlane", "v_writelane", "v_readfirstlane")):
        return "mov"
    if op.startswith("v_cvt"):
        return "cvt"
    if op.startswith(("v_fma_f32", "v_fmac_f32", "v_mul_f32", "v_add_f32", "v_sub_f32", "v_mac_f32")):
        return "f32"
    if op.startswith("v_"):
        return "valu-int"
    return "other"


def main():
    path, kname = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(kname), l) or (l.startswith("_Z") and kname in l.split(":")[0]))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    segs, cur = [], ("prologue", collections.Counter())
    for l in lines[start:end]:
        t = l.strip()
        m = re.search(r";\s*PHASE\s+(\d+)", t)
        if m:
            segs.append(cur)
            cur = (int(m.group(1)), collections.Counter())
            continue
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        cur[1][klass(op, t)] += 1
        cur[1]["_total"] += 1
    segs.append(cur)
    info = None
    if len(sys.argv) > 4:
        info = (int(sys.argv[3], 16), int(sys.argv[4], 16))
    tot = collections.Counter()
    kinds = collections.defaultdict(collections.Counter)
    phi = -1
    for name, c in segs:
        tot.update(c)
        if name == "prologue":
            kinds["prologue"].update(c)
            continue
        phi += 1
        if info:
            is_info = (info[phi >> 6] >> (phi & 63)) & 1
            kind = ("info" if is_info else "frozen") + ("+recompute" if phi % 16 == 0 else "")
        else:
            kind = f"t{name}"
        kinds[kind].update(c)
    kinds["(last segment incl. epilogue)"] = segs[-1][1]
    cls = sorted({k for c in kinds.values() for k in c if k != "_total"})
    print(f"{'kind':34s} {'n':>4s} {'total':>7s} " + " ".join(f"{k[:10]:>10s}" for k in cls))
    nk = collections.Counter()
    phi = -1
    for name, _ in segs:
        if name == "prologue":
            continue
        phi += 1
        if info:
            is_info = (info[phi >> 6] >> (phi & 63)) & 1
            nk[("info" if is_info else "frozen") + ("+recompute" if phi % 16 == 0 else "")] += 1
    for k, c in kinds.items():
        print(f"{k:34s} {nk.get(k, 0):4d} {c['_total']:7d} " + " ".join(f"{c[x]:10d}" for x in cls))
    print(f"{'TOTAL':34s} {'':4s} {tot['_total']:7d} " + " ".join(f"{tot[x]:10d}" for x in cls))


if __name__ == "__main__":
    main()
