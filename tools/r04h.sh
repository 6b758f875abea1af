#!/bin/bash
# Round-4 GPU pass h: 4-deep DL-SCL pipeline (config 3), stashed side streams; tests of the
# pipelined paths, config-3 sweep timing, bench line.
set -o pipefail
tag=${1:-r04h}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fer.py tests/test_gpu_long.py -x -q --timeout 250 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/${tag}_tests.log | head -30; exit 1; }
timeout -k 10 300 python3 tools/config3_run.py | grep "config 3" || exit 1
timeout -k 10 300 python3 tools/config3_run.py 1000000 5.0 5.0 | grep "config 3" || exit 1
timeout -k 10 300 python3 tools/long_bench.py > gpurun_out/${tag}_long_bench.txt 2>&1; grep "frames/s" gpurun_out/${tag}_long_bench.txt
timeout -k 10 400 python3 bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][-1])
print('value', round(d['value']/1e6,1), 'ms', round(d['ms_per_step'],3), 'launch', round(d['roofline']['avg_launch_ms'],3), 'parity', d['parity']['mismatches'], '/', d['parity']['frames'])
for k,v in (d['extra_configs'] or {}).items(): print(k, round(v['value']/1e6,1), v.get('ms_per_step'), v.get('point_5db'))
"
