#!/bin/bash
# Round-4 GPU pass s2: side chain + every chain beside a later baseline screened (L = 4 and 8).
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_baseline_configs.py tests/test_gpu_fer.py tests/test_gpu_screening.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04s2_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04s2_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r04s2_tests.log | head -30; exit 1; }
echo "config 4:"; timeout -k 10 300 bash tools/dl_tune.sh 2 - dl_screen=2 || exit 1
for r in 1 2; do
  for t in "" "dl_screen=2"; do
    timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 6.5 $t | grep "config 3" || exit 1
  done
done
timeout -k 10 200 python3 tools/config3_run.py 1000000 5.0 5.0 | grep "config 3" || exit 1
