#!/bin/bash
# Interleaved A/B of handle knobs (pscl_set_tuning) on one workload, `rounds` times:
#   bash tools/knob_ab.sh <tag> <rounds> <workload> "<k=v[,k=v]|->" ...
# workloads:  sweep  config-3 sweep, L = 8, 4.0-6.5 dB, 10^6 frames/point (tools/config3_run.py)
#             p5     its 5 dB point alone
#             c4     config 4: bench.py --list 4 --retries 8 (beta_M4, pipelined, 10 steps)
#             head   the headline: bench.py --extra none --no-cpu-baseline (10 steps)
# (replaces round 6's tx_ab.sh / fp_ab.sh / c3_knob_ab.sh / c4_tune.sh; library variants: ab_bench.sh)
set -o pipefail
tag=$1; rounds=$2; wl=$3; shift 3
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 $rounds); do
  i=0
  for t in "$@"; do
    i=$((i+1)); log=$out/${wl}_$i.$r.log
    case $wl in
      sweep) cmd="python3 tools/config3_run.py 1000000 4.0 6.5 $t" ;;
      p5) cmd="python3 tools/config3_run.py 1000000 5.0 5.0 $t" ;;
      c4|head)
        arg=""; [ "$t" != "-" ] && arg="--tune $t"
        if [ $wl = c4 ]; then cmd="python3 bench.py --list 4 --retries 8 --steps 10 --warmup 2 --no-cpu-baseline --extra none $arg ${KNOB_AB_EXTRA:-}"
        else cmd="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --extra none $arg ${KNOB_AB_EXTRA:-}"; fi ;;
      *) echo "unknown workload $wl"; exit 2 ;;
    esac
    timeout -k 10 200 $cmd > $log 2>&1 || { echo "$wl $t failed"; tail -5 $log; exit 1; }
    res=$(python3 -c "
import json
for l in open('$log'):
    if l.startswith('{'):
        d = json.loads(l); print(round(d['ms_per_step'], 3), 'ms/step', round(d['value'] / 1e6, 1), 'M frames/s')
    elif 'frames/s' in l:
        print(l.strip().split(' in ')[-1])" | tail -1)
    echo "$wl $t: $res"
  done
done
