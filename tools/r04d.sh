#!/bin/bash
# Round-4 GPU pass d: DL-SCL baseline kernel A/B (config 4, config 3 points), long-code kernels
# (timing + rocprofv3 kernel stats), PMC passes of the headline build.
set -o pipefail
tag=${1:-r04d}
mkdir -p gpurun_out
echo "config 4 (prod = DL baseline on the 2-lanes kernel, dllane = lane-per-path):"
timeout -k 10 400 bash tools/ab_bench.sh "prod dllane" 2 --list 4 --retries 8 || exit 1
for v in prod dllane; do
  echo "config 3 points ($v):"
  PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 300 python3 tools/sweep_timing.py 8 1000000 1048576 1 4.0,5.0,6.0 2>&1 | grep "M=8" || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_long_${tag} -o long -- python3 tools/long_bench.py > gpurun_out/${tag}_long_bench.txt 2>&1 || { tail -20 gpurun_out/${tag}_long_bench.txt; exit 1; }
grep "frames/s" gpurun_out/${tag}_long_bench.txt
find gpurun_out/prof_long_${tag} -name "*kernel_stats.csv" | head -1 | xargs -I{} python3 -c "
import csv,sys
rows=list(csv.DictReader(open('{}')))
for r in rows[:12]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,2), 'ms total')"
bash tools/profile_pmc.sh ${tag} || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_${tag} 1000000 --json > gpurun_out/${tag}_pmc_summary.txt 2>&1; tail -30 gpurun_out/${tag}_pmc_summary.txt
