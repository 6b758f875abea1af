#!/bin/bash
# Interleaved timing of DL-SCL (config 4: L=4, 8 retries, beta_M4) under handle tuning knobs:
#   bash tools/dl_tune.sh <rounds> "<knobs 1>" "<knobs 2>" ...   [DLT_ARGS="--list 8 ..." extra bench args]
# each knob string is bench.py's --tune value (k=v[,k=v], pscl_set_tuning), or "-" for the defaults
set -o pipefail
rounds=$1; shift
mkdir -p gpurun_out/dltune
for r in $(seq 1 $rounds); do
  i=0
  for cfg in "$@"; do
    i=$((i + 1))
    tn=""; [ "$cfg" != "-" ] && tn="--tune $cfg"
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --extra none --list 4 --retries 8 $DLT_ARGS $tn > gpurun_out/dltune/$i.$r.log 2>&1 || { echo "[$cfg] failed"; tail -5 gpurun_out/dltune/$i.$r.log; exit 1; }
    echo "[$cfg] $(grep '^{' gpurun_out/dltune/$i.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["dl_scl"]["frame_errors"] if d.get("dl_scl") else None, (d.get("parity") or {}).get("mismatches"))')"
  done
done
