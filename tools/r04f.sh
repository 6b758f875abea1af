#!/bin/bash
# Round-4 GPU pass f: long-code tests and timing with the LDS-resident exact re-decode.
set -o pipefail
tag=${1:-r04f}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_long.py tests/test_gpu_lane_long.py -x -q -s --timeout 250 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; grep -E "deferred|passed|failed" gpurun_out/${tag}_tests.log | tail -14
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/${tag}_tests.log | head -30; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_long_${tag} -o long -- python3 tools/long_bench.py > gpurun_out/${tag}_long_bench.txt 2>&1 || { tail -20 gpurun_out/${tag}_long_bench.txt; exit 1; }
grep "frames/s" gpurun_out/${tag}_long_bench.txt
f=$(find gpurun_out/prof_long_${tag} -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:14]: print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,2), 'ms total')"
timeout -k 10 300 python3 tools/long_bench.py --dl > gpurun_out/${tag}_long_dl.txt 2>&1; cat gpurun_out/${tag}_long_dl.txt | grep -v amdgpu.ids
