"""Summarise rocprofv3 PMC passes (tools/profile_pmc.sh output) for the decode kernel.

    python tools/pmc_summary.py gpurun_out/pmc_<tag> [frames_per_launch] [--json] [--write KEY]

Prints per-launch averages and derived figures, and (with --json) the HBM traffic entry
bench.py reads from profiles/pmc_traffic.json.  Corrections follow MI355X_MICROARCH.md
(HBM section): FETCH_SIZE/WRITE_SIZE are in KiB; gfx950 FETCH_SIZE reports half the bytes of
wide coalesced reads, so it is doubled; WRITE_SIZE is taken as reported.
"""
import collections
import csv
import json
import sys
from pathlib import Path


def load(d):
    """Per-dispatch averages of the dominant decode kernel (with screening, the screening
    kernel; the exact re-decode of the deferred frames is a separate, near-empty launch)."""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(Path(d).glob("p*/pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if any(k in r["Kernel_Name"] for k in ("scl_decode_kernel", "scl128_kernel", "scl_lane_kernel",
                                                    "scl_lane_long_kernel")):
                agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not agg:
        return {}
    per = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}
    main = max(per, key=lambda k: sum(per[k].values()))
    return per[main]


def main():
    d = sys.argv[1]
    frames = float(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 1e6
    c = load(d)
    for k in sorted(c):
        print(f"{k:28s} {c[k]:.6g}")
    out = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fetch = 2 * c["FETCH_SIZE"] * 1024
        write = c["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = fetch + write
        out["fetch_bytes_corrected"] = fetch
        out["write_bytes"] = write
        print(f"HBM bytes/launch (2*FETCH+WRITE) = {fetch + write:.4g}  ({(fetch + write) / frames:.1f} B/frame)")
    if "SQ_WAVES" in c:
        w = c["SQ_WAVES"]
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
            if k in c:
                print(f"{k} per wave = {c[k] / w:.0f}")
    if "GRBM_GUI_ACTIVE" in c:
        print(f"GRBM_GUI_ACTIVE = {c['GRBM_GUI_ACTIVE']:.4g}")
    for k, name in (("SQ_INSTS_VALU", "valu"), ("SQ_INSTS_SALU", "salu"), ("SQ_INSTS_LDS", "lds")):
        if k in c:
            out[f"{name}_instr_per_frame"] = round(c[k] / frames, 2)
    if "SQ_ACTIVE_INST_VALU" in c and "GRBM_GUI_ACTIVE" in c:
        # quad-cycles summed over waves, x4 -> cycles; 1024 SIMDs; GRBM counts per XCD (8)
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        out["valu_active_frac"] = round(c["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * cyc), 4)
        out["valu_active_frac_def"] = "SQ_ACTIVE_INST_VALU*4 / (1024 SIMDs * GRBM_GUI_ACTIVE/8)"
        if "SQ_INSTS_VALU" in c:
            out["cycles_per_valu_instr"] = round(1024 * cyc / c["SQ_INSTS_VALU"], 3)
            print(f"SIMD cycles per VALU instruction = {out['cycles_per_valu_instr']}")
    mix = {k[len("SQ_INSTS_VALU_"):].lower(): round(c[k] / frames, 1) for k in c if k.startswith("SQ_INSTS_VALU_")}
    if mix:
        out["valu_mix_per_frame"] = mix
    if "SQ_LDS_BANK_CONFLICT" in c:
        out["lds_bank_conflict_cycles"] = c["SQ_LDS_BANK_CONFLICT"]
        if "SQ_LDS_IDX_ACTIVE" in c and c["SQ_LDS_IDX_ACTIVE"] > 0:
            out["lds_bank_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
            out["lds_bank_conflict_frac_def"] = "SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (cycles)"
            print(f"LDS bank conflict cycles / LDS active cycles = {out['lds_bank_conflict_frac']}")
    for k in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"):
        if k in c:
            out[k.lower()] = c[k]
    if "GRBM_GUI_ACTIVE" in c:
        out["grbm_gui_active"] = c["GRBM_GUI_ACTIVE"]
    # the library the passes ran (its embedded source hash): bench.py only uses an entry
    # measured on the build it times
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from polar_code_amd import build

    out["build_hash"] = build.library_hash()
    out["source"] = f"{d}: rocprofv3 --pmc passes (tools/profile_pmc.sh), one counter group per pass"
    if "--json" in sys.argv:
        print(json.dumps(out))
    if "--write" in sys.argv:
        key = sys.argv[sys.argv.index("--write") + 1]
        p = Path(__file__).resolve().parent.parent / "profiles" / "pmc_traffic.json"
        db = json.loads(p.read_text()) if p.exists() else {}
        db[key] = out
        p.write_text(json.dumps(db, indent=1, sort_keys=True) + "\n")
        print(f"wrote {key} to {p}")


if __name__ == "__main__":
    main()
