#!/bin/bash
# Round-4 GPU check: screening + channel tests, lane-kernel A/B, bench line, full GPU suite,
# config-3 trace.
set -o pipefail
tag=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lane_long.py tests/test_gpu_screening.py tests/test_gpu_channel.py -x -q -s --timeout 250 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log; grep -E "scan:|screening tail" gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/${tag}_tests.log | head -20; exit 1; }
for L in 8 4; do PSCL_LANE_STATS=1 PSCL_LIB_PATH=tools/_variant/lib_lanestats.so timeout -k 10 120 python3 tools/fastpath_stats.py $L 5.0; done
timeout -k 10 400 bash tools/ab_bench.sh "prod noswap nolane reltail" 2 || exit 1
echo "L=4:"; timeout -k 10 300 bash tools/ab_bench.sh "prod creg4 nolane" 2 --list 4 || exit 1
echo "config 4:"; timeout -k 10 400 bash tools/ab_bench.sh "prod nofma nolane" 2 --list 4 --retries 8 || exit 1
bash tools/quick_gpu.sh ${tag} || exit 1
timeout -k 10 300 python -u tools/long_bench.py > gpurun_out/${tag}_long_bench.txt 2>&1; cat gpurun_out/${tag}_long_bench.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/${tag}_gpu_suite.log 2>&1
rc=$?; tail -5 gpurun_out/${tag}_gpu_suite.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/${tag}_gpu_suite.log | head -30; exit 1; }
bash tools/profile_sim_trace.sh ${tag} 4.0,5.0
