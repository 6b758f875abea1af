#!/bin/bash
# Round-4 GPU pass q: lane-per-path forced-bit screening kernel for the DL-SCL retry decodes.
set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_fer.py -x -q --timeout 250 --timeout-method thread -k "retry_loop_equals" > gpurun_out/r04q_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04q_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r04q_tests.log | head -30; exit 1; }
for r in 1 2; do
  for t in "" "dl_screen=1" "dl_retry_lane=2" "dl_screen=2"; do
    timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 6.5 $t | grep "config 3" || exit 1
  done
done
for e in 4.0 5.0 6.0; do
  for t in "" "dl_screen=1" "dl_screen=2"; do
    timeout -k 10 200 python3 tools/config3_run.py 1000000 $e $e $t | grep "config 3" || exit 1
  done
done
echo "config 4:"; timeout -k 10 300 bash tools/dl_tune.sh 2 - dl_screen=1 || exit 1
