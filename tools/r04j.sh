#!/bin/bash
# Round-4 GPU pass j: Layout128 stride padding for narrow frames (L = 4 two-lanes kernel): tests,
# A/B on config 4 (baseline + FS retry decodes at L = 4), PMC of config 4.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_screening.py tests/test_gpu_parity.py tests/test_gpu_fer.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r04j_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04j_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r04j_tests.log | head -30; exit 1; }
echo "config 4:"; timeout -k 10 400 bash tools/ab_bench.sh "prod pad0" 3 --list 4 --retries 8 || exit 1
bash tools/kernel_pmc.sh c4pad python3 bench.py --list 4 --retries 8 --steps 2 --warmup 1 --no-cpu-baseline --extra none > gpurun_out/r04j_c4_pmc.txt 2>&1 || { tail -5 gpurun_out/r04j_c4_pmc.txt; exit 1; }
head -12 gpurun_out/r04j_c4_pmc.txt
