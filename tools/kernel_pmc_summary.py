"""Per-kernel summary of tools/kernel_pmc.sh passes: counters averaged per dispatch, grouped by
kernel name (template arguments kept), with the derived figures of MI355X_MICROARCH.md's HBM
section (FETCH_SIZE doubled on gfx950, KiB units), VALU / LDS per wave, VALU-active fraction over
the dispatch's GRBM cycles, LDS bank-conflict fraction.

    python tools/kernel_pmc_summary.py <dir> [--json]
"""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(d + "/p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, cs in agg.items():
    c = {n: sum(v) / len(v) for n, v in cs.items()}
    e = {"dispatches": max(len(v) for v in cs.values())}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        e["hbm_bytes"] = 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
    if "SQ_WAVES" in c and c["SQ_WAVES"]:
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if n in c:
                e[n.lower() + "_per_wave"] = round(c[n] / c["SQ_WAVES"], 1)
        e["waves"] = c["SQ_WAVES"]
    if "GRBM_GUI_ACTIVE" in c:
        e["gpu_us"] = round(c["GRBM_GUI_ACTIVE"] / 8 / 2.4e3, 1)  # per-XCD count, ~2.4 GHz
        if "SQ_ACTIVE_INST_VALU" in c:
            e["valu_active_frac"] = round(c["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * c["GRBM_GUI_ACTIVE"] / 8), 4)
    if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
        e["lds_bank_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
    if "SQ_WAIT_INST_ANY" in c and c.get("SQ_WAVE_CYCLES"):
        e["wait_inst_frac"] = round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4)
    e["counters"] = {n: round(v, 1) for n, v in c.items()}
    out[k] = e
for k, e in sorted(out.items(), key=lambda x: -x[1].get("gpu_us", 0)):
    print(k[:110])
    print("   ", {n: v for n, v in e.items() if n != "counters"})
if "--json" in sys.argv:
    print(json.dumps(out))
