#!/bin/bash
# Round-4 GPU pass g: config-3 sweep timing and its host/kernel trace (where the wall time goes).
set -o pipefail
tag=${1:-r04g}
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/config3_run.py | grep "config 3"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/c3trace_${tag}
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $out -o c3 -- python3 tools/config3_run.py > $out.log 2>&1 || { tail -5 $out.log; exit 1; }
grep "config 3" $out.log
python3 tools/api_gaps.py $out 150 > gpurun_out/${tag}_c3_gaps.txt 2>&1; tail -60 gpurun_out/${tag}_c3_gaps.txt
