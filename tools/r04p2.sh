#!/bin/bash
# Round-4 GPU pass p2: per-dispatch dl_post_kernel time under post-pass ablations (timing only),
# from rocprofv3 kernel traces of the config-4 bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in prod pa2 pa4 pa8; do
  out=gpurun_out/p2_$v; mkdir -p $out
  PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o trace -- python3 bench.py --list 4 --retries 8 --steps 5 --warmup 1 --no-cpu-baseline --extra none > $out/bench.log 2>&1 || { echo "$v failed"; tail -3 $out/bench.log; exit 1; }
  f=$(ls $out/*kernel_stats.csv $out/*/*kernel_stats.csv 2>/dev/null | head -1)
  echo "$v: $(grep -E 'dl_post_kernel|scl_lane_kernel<4, 1, true>|scl128_kernel<4, false, false, true' $f | cut -d, -f1-4 | tr '\n' ' ')"
done
