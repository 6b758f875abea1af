#!/bin/bash
# Round-4 GPU pass p: adaptive screening of DL-SCL retry decodes (chain size threshold).
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_fer.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r04p_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04p_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r04p_tests.log | head -30; exit 1; }
for r in 1 2; do
  for t in "dl_screen=2" "" "dl_screen_min=12288" "dl_screen_min=49152"; do
    timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 6.5 $t | grep "config 3" || exit 1
  done
done
for t in "dl_screen=2" "" "dl_screen_min=12288"; do
  timeout -k 10 200 python3 tools/config3_run.py 1000000 4.5 4.5 $t | grep "config 3" || exit 1
done
echo "config 4 (default vs never):"; timeout -k 10 300 bash tools/dl_tune.sh 2 - dl_screen=2 || exit 1
