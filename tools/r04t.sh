#!/bin/bash
# Round-4 GPU pass t: post-pass ablations (timing only; outputs invalid) on config 4 and the
# standalone config-3 5 dB point, then a kernel trace of the 5 dB point (product build).
set -o pipefail
bash tools/ab_bench.sh "prod pa1 pa2 pa4 pa8 pa15" 2 --list 4 --retries 8 || exit 1
for r in 1 2; do
  for v in prod pa2 pa4 pa8 pa15; do
    echo -n "$v "; PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 200 python3 tools/config3_run.py 1000000 5.0 5.0 | grep "config 3" || exit 1
  done
done
bash tools/profile_sim_trace.sh r04t 5.0 > gpurun_out/r04t_trace.txt 2>&1 || { tail -5 gpurun_out/r04t_trace.txt; exit 1; }
head -80 gpurun_out/r04t_trace.txt
