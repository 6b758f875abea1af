#!/bin/bash
# Round-4 GPU pass m: lane kernel on the NR (128,88) rate-matched code (config 5): tests + A/B.
set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_gpu_screening.py tests/test_gpu_nr_ber.py tests/test_gpu_baseline_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04m_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04m_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r04m_tests.log | head -30; exit 1; }
echo "config 5:"; timeout -k 10 400 bash tools/ab_bench.sh "nrlane prod" 3 --nr-E 256 || exit 1
