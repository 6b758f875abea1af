#!/bin/bash
# Round-4 GPU pass b32: narrow post pass with beta staged in LDS as fp32 (prod) vs through L2 (b64).
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_fer.py tests/test_gpu_baseline_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04b32_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04b32_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r04b32_tests.log | head -30; exit 1; }
bash tools/ab_bench.sh "prod b64" 3 --list 4 --retries 8 || exit 1
for r in 1 2; do
  for v in prod b64; do
    echo -n "$v "; PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 6.5 | grep "config 3" || exit 1
  done
done
