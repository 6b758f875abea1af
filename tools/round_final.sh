#!/bin/bash
# Round-final GPU pass on the frozen build: full GPU suite, smoke, default bench line,
# rocprofv3 kernel stats + PMC passes of the headline, long codes, config-3 sweep, kernel PMC of
# configs 3 and 4.
#   bash tools/round_final.sh <tag>
set -o pipefail
tag=${1:?tag}
bash tools/gpu_round.sh ${tag} || exit 1
tail -3 gpurun_out/${tag}_gpu_tests.log
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][-1])
print('value', round(d['value']/1e6,1), 'ms', round(d['ms_per_step'],3), 'parity', d['parity']['mismatches'], '/', d['parity']['frames'])
for k,v in (d['extra_configs'] or {}).items(): print(k, round(v['value']/1e6,1), v.get('ms_per_step'))
"
tail -4 gpurun_out/${tag}_pmc_summary.txt
timeout -k 10 300 python3 tools/long_bench.py > gpurun_out/${tag}_long_bench.txt 2>&1; grep "frames/s" gpurun_out/${tag}_long_bench.txt
timeout -k 10 300 python3 tools/config3_run.py | grep "config 3"
timeout -k 10 300 python3 tools/config3_run.py 1000000 5.0 5.0 | grep "config 3"
bash tools/kernel_pmc.sh ${tag}_c3 python3 tools/config3_run.py 1000000 5.0 5.0 > gpurun_out/${tag}_c3_pmc.txt 2>&1 || { tail -5 gpurun_out/${tag}_c3_pmc.txt; exit 1; }
bash tools/kernel_pmc.sh ${tag}_c4 python3 bench.py --list 4 --retries 8 --steps 2 --warmup 1 --no-cpu-baseline --extra none > gpurun_out/${tag}_c4_pmc.txt 2>&1 || { tail -5 gpurun_out/${tag}_c4_pmc.txt; exit 1; }
echo final-done
