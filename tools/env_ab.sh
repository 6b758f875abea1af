#!/bin/bash
# Interleaved A/B timing of one environment variable: bash tools/env_ab.sh VAR "<values>" <rounds> [bench args]
# (prints ms_per_step of each run; e.g. tools/env_ab.sh PSCL_DL_SPLIT "1 2" 3 --list 4 --retries 8)
set -o pipefail
var=$1; vals=$2; rounds=${3:-3}; shift 3
mkdir -p gpurun_out/envab
for r in $(seq 1 $rounds); do
  for v in $vals; do
    env "$var=$v" timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --extra none "$@" > gpurun_out/envab/$v.$r.log 2>&1 || { echo "$v failed"; exit 1; }
    echo "$var=$v $(grep '^{' gpurun_out/envab/$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("parity"))')"
  done
done
