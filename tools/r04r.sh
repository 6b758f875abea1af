#!/bin/bash
# Round-4 GPU pass r: lane FS retry decodes, per-L screening default; oracle checks at size.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline_configs.py tests/test_gpu_fer.py -x -v --timeout 300 --timeout-method thread -k "screened or config4 or retry_loop_equals or config3 or pipelined" > gpurun_out/r04r_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r04r_tests.log | tail -30
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/r04r_tests.log | head -30; exit 1; }
for r in 1 2; do
  for t in "" "dl_screen_min=4096" "dl_screen_min=24576"; do
    timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 6.5 $t | grep "config 3" || exit 1
  done
done
