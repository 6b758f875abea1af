#!/bin/bash
# Dynamic instruction counts and timing of the ablation builds (tools/ablate.py build first).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ablate
mkdir -p $out
for m in ${MASKS:-0 1 2 4 8 16 7}; do
    timeout -k 10 200 python3 tools/ablate.py run $m ${L:-8} > $out/t$m.log 2>&1 || { echo "time $m failed"; exit 1; }
    timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $out/p$m -o pmc -- \
        python3 tools/ablate.py run $m ${L:-8} > $out/p$m.log 2>&1 || { echo "pmc $m failed"; exit 1; }
    python3 - $out/p$m $m <<'PY'
import csv, glob, sys
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
rows = [r for r in rows if "scl128_kernel" in r.get("Kernel_Name", "")]
tot = {}
for r in rows:
    tot.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = tot.setdefault(r["Dispatch_Id"], {}).get(r["Counter_Name"], 0) + float(r["Counter_Value"])
last = tot[sorted(tot, key=int)[-1]]
w = last["SQ_WAVES"]
print(f"mask={sys.argv[2]} VALU/wave={last['SQ_INSTS_VALU']/w:.0f} SALU/wave={last['SQ_INSTS_SALU']/w:.0f}")
PY
    cat $out/t$m.log | grep ablate
done
