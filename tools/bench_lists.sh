#!/bin/bash
# Short bench of every list size (no CPU baseline); one JSON summary line per L.
#   bash tools/bench_lists.sh [extra bench args...]
set -o pipefail
mkdir -p gpurun_out
for L in 8 4 2 1; do
    timeout -k 10 200 python3 bench.py --list $L --steps 5 --warmup 1 --no-cpu-baseline --extra none "$@" > gpurun_out/bl_$L.log 2>&1 || { echo "L=$L failed"; exit 1; }
    grep '^{' gpurun_out/bl_$L.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('L=$L', round(d['value']/1e6,2), 'Mframes/s', round(r['avg_launch_ms'],3), 'ms/launch', 'fer', d['fer']['fer'])"
done
