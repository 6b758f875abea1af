#!/bin/bash
# Quick GPU check of the current build: screening/parity tests, screening rate, bench line.
#   bash tools/quick_gpu.sh <tag> [ab-variants]
set -o pipefail
tag=${1:-q}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_screening.py tests/test_gpu_parity.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
grep "screening tail" gpurun_out/${tag}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.log; exit 1; }
python -c "
import json; d=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][-1])
print('value', round(d['value']/1e6,1), 'ms', round(d['ms_per_step'],3), 'launch', round(d['roofline']['avg_launch_ms'],3), 'parity', d['parity']['mismatches'], '/', d['parity']['frames'], 'fer', d['fer']['frame_errors'])
for k,v in (d['extra_configs'] or {}).items(): print(k, round(v['value']/1e6,1), round(v['ms_per_step'],3), v['parity']['mismatches'])
"
if [ -n "$2" ]; then timeout -k 10 400 bash tools/ab_bench.sh "$2" 3; fi
