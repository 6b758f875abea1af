#!/bin/bash
# Fused-TX A/B on the config-3 sweep (tools/config3_run.py, L = 8, 10^6 frames per point): the
# separate TX launch (tx_fused=2) against the fused one (tx_fused=1), alternating, `rounds` times,
# the 6-point sweep and the 5 dB point.   bash tools/tx_ab.sh <tag> [rounds]
set -o pipefail
tag=$1; rounds=${2:-2}
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 $rounds); do
  for v in 2 1; do
    timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 6.5 tx_fused=$v > $out/sweep_$v.$r.log 2>&1 || { echo "sweep $v failed"; tail -5 $out/sweep_$v.$r.log; exit 1; }
    timeout -k 10 200 python3 tools/config3_run.py 1000000 5.0 5.0 tx_fused=$v > $out/p5_$v.$r.log 2>&1 || { echo "5dB $v failed"; tail -5 $out/p5_$v.$r.log; exit 1; }
    echo "tx_fused=$v: $(grep 'frames/s' $out/sweep_$v.$r.log | tail -1 | sed 's/.*in/in/') | 5 dB $(grep 'frames/s' $out/p5_$v.$r.log | tail -1 | sed 's/.*in/in/')"
  done
done
