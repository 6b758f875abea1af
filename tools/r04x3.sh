#!/bin/bash
# Round-4 GPU pass x3: the pipelined DL-SCL equality test, committed build (base) vs side chain (side), 4 runs each.
set -o pipefail
for r in 1 2 3 4; do
  for v in base side; do
    PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fer.py -x -q --timeout 250 --timeout-method thread -k "pipelined_dlscl_calls_equal" > gpurun_out/r04x3_${v}_$r.log 2>&1
    echo "$v run $r rc=$? $(grep -cE '^E ' gpurun_out/r04x3_${v}_$r.log) $(grep -E '^E .*(ACTUAL|DESIRED)' -A1 gpurun_out/r04x3_${v}_$r.log | tr '\n' ' ' | cut -c1-300)"
  done
done
