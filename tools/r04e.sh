#!/bin/bash
# Round-4 GPU pass e: long-code kernels (timing + rocprofv3 kernel stats), the default bench line,
# PMC passes of the headline build.
set -o pipefail
tag=${1:-r04e}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_long_${tag} -o long -- python3 tools/long_bench.py > gpurun_out/${tag}_long_bench.txt 2>&1 || { tail -20 gpurun_out/${tag}_long_bench.txt; exit 1; }
grep "frames/s" gpurun_out/${tag}_long_bench.txt
f=$(find gpurun_out/prof_long_${tag} -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:12]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,2), 'ms total')"
timeout -k 10 400 python3 bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${tag}_bench.log') if l.startswith('{')][-1])
print('value', round(d['value']/1e6,1), 'ms', round(d['ms_per_step'],3), 'launch', round(d['roofline']['avg_launch_ms'],3), 'parity', d['parity']['mismatches'], '/', d['parity']['frames'])
for k,v in (d['extra_configs'] or {}).items(): print(k, round(v['value']/1e6,1), v.get('ms_per_step'), v.get('point_5db'))
"
bash tools/profile_pmc.sh ${tag} || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_${tag} 1000000 --json > gpurun_out/${tag}_pmc_summary.txt 2>&1; tail -30 gpurun_out/${tag}_pmc_summary.txt
