#!/bin/bash
# Kernel timelines of the config-3 5 dB point with the post pass separate (2) and fused (1).
#   bash tools/fp_trace.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag; mkdir -p $out
for v in 2 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/t$v -o t -- python3 tools/config3_run.py 1000000 5.0 5.0 dl_fused_post=$v > $out/t$v.log 2>&1 || { echo "trace $v failed"; tail -5 $out/t$v.log; exit 1; }
  python3 tools/dl_timeline.py $out/t$v 4 0 > $out/timeline_$v.txt 2>&1 || true
  echo "== dl_fused_post=$v"; cat $out/timeline_$v.txt | head -70
done
