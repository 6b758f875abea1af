#!/bin/bash
# Round-4 GPU pass x2: side-chain timing, then the pipelined-equality test alone (twice).
set -o pipefail
echo "config 4:"; timeout -k 10 300 bash tools/dl_tune.sh 2 - dl_screen=1 || exit 1
for r in 1 2; do
  for t in "" "dl_screen=1"; do
    timeout -k 10 200 python3 tools/config3_run.py 1000000 5.0 5.0 $t | grep "config 3" || exit 1
  done
done
for r in 1 2; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fer.py -x -q --timeout 250 --timeout-method thread -k "pipelined_dlscl_calls_equal" > gpurun_out/r04x2_t$r.log 2>&1; echo "test run $r rc=$?"; grep -E "^E  .*(ACTUAL|DESIRED|array)|passed|failed" gpurun_out/r04x2_t$r.log | head -8
done
