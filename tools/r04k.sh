#!/bin/bash
# Round-4 GPU pass k: error counters aggregated per wavefront / workgroup (counting launches
# capped, atomics once per wavefront): tests, A/B against the per-frame-atomics build (old).
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fer.py tests/test_gpu_channel.py tests/test_gpu_lane_long.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r04k_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04k_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/r04k_tests.log | head -30; exit 1; }
echo "L=8 5 dB:"; timeout -k 10 300 bash tools/ab_bench.sh "prod old" 2 || exit 1
echo "L=8 4 dB:"; timeout -k 10 300 bash tools/ab_bench.sh "prod old" 2 --ebno 4.0 || exit 1
echo "config 4:"; timeout -k 10 300 bash tools/ab_bench.sh "prod old" 2 --list 4 --retries 8 || exit 1
echo "config 5:"; timeout -k 10 300 bash tools/ab_bench.sh "prod old" 2 --nr-E 256 || exit 1
for v in prod old; do echo "config 3 ($v):"; PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 300 python3 tools/config3_run.py | grep "config 3" || exit 1; done
for v in prod old; do echo "config 3 ($v):"; PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 300 python3 tools/config3_run.py | grep "config 3" || exit 1; done
