#!/bin/bash
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_screening.py tests/test_gpu_fer.py tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r04n_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04n_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r04n_tests.log | head -30; exit 1; }
echo "L=8 5 dB:"; timeout -k 10 400 bash tools/ab_bench.sh "prod old" 4 || exit 1
echo "L=4:"; timeout -k 10 300 bash tools/ab_bench.sh "prod old" 2 --list 4 || exit 1
