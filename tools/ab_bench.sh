#!/bin/bash
# Interleaved A/B timing of library variants: bash tools/ab_bench.sh "<libs>" <rounds> [bench args]
set -o pipefail
libs=$1; rounds=${2:-3}; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 $rounds); do
  for v in $libs; do
    PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --extra none "$@" > gpurun_out/ab/$v.$r.log 2>&1 || { echo "$v failed"; exit 1; }
    echo "$v $(grep '^{' gpurun_out/ab/$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["roofline"]["avg_launch_ms"],3), round(d["ms_per_step"],3), d["parity"]["mismatches"] if d.get("parity") else None)')"
  done
done
