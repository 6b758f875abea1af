#!/bin/bash
# rocprofv3 kernel traces of the DL-SCL bench (config 4) for library variants; per-kernel mean
# times of each.   bash tools/dl_variant_trace.sh <tag> "<variants>"   ("prod" = the product)
set -o pipefail
tag=$1; vars=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in $vars; do
  out=gpurun_out/dlv_${tag}_$v
  mkdir -p "$out"
  if [ "$v" = prod ]; then lp=""; else lp=tools/_variant/lib_$v.so; fi
  PSCL_LIB_PATH=$lp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o trace -- \
      python3 bench.py --list 4 --retries 8 --steps 3 --warmup 1 --no-cpu-baseline --extra none > "$out/bench.log" 2>&1 || { echo "$v failed"; tail -5 "$out/bench.log"; exit 1; }
  python3 - "$out" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + "/trace_kernel_stats.csv")))
for r in rows:
    n = r["Name"]
    if "dl_post" in n or "true, 1, false" in n:
        print(sys.argv[2], n[:60], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us avg", round(float(r["MaxNs"]) / 1000, 1), "max")
PY
done
