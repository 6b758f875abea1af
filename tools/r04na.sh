#!/bin/bash
# Round-4 GPU pass na: wide post pass for chains running alone (prod) vs narrow (na1).
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_fer.py -x -q --timeout 300 --timeout-method thread -k "pipelined or config3 or simulate or sweep" > gpurun_out/r04na_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r04na_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r04na_tests.log | head -30; exit 1; }
for r in 1 2 3; do
  for v in prod na1; do
    echo -n "$v "; PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 200 python3 tools/config3_run.py 1000000 5.0 5.0 | grep "config 3" || exit 1
  done
done
for v in prod na1; do
  echo -n "$v "; PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 6.5 | grep "config 3" || exit 1
done
bash tools/ab_bench.sh "prod na1" 1 --list 4 --retries 8 || exit 1
