#!/bin/bash
# Interleaved timing of DL-SCL (config 4: L=4, 8 retries, beta_M4) under environment settings:
#   bash tools/dl_tune.sh <rounds> "<env settings 1>" "<env settings 2>" ...
# each settings string is a space-separated list of VAR=value (or "-" for none)
set -o pipefail
rounds=$1; shift
mkdir -p gpurun_out/dltune
for r in $(seq 1 $rounds); do
  i=0
  for cfg in "$@"; do
    i=$((i + 1))
    envs=""; [ "$cfg" != "-" ] && envs="$cfg"
    env $envs timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --extra none --list 4 --retries 8 > gpurun_out/dltune/$i.$r.log 2>&1 || { echo "[$cfg] failed"; tail -5 gpurun_out/dltune/$i.$r.log; exit 1; }
    echo "[$cfg] $(grep '^{' gpurun_out/dltune/$i.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["dl_scl"]["frame_errors"] if d.get("dl_scl") else None, d["parity"]["mismatches"])')"
  done
done
