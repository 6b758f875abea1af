#!/bin/bash
# Round-4 GPU pass v: post-pass occupancy hint / unroll variants (post_pairs = 2 default in all).
set -o pipefail
bash tools/ab_bench.sh "prod u16 w2 w2u16" 2 --list 4 --retries 8 || exit 1
for r in 1 2; do
  for v in prod u16 w2 w2u16; do
    echo -n "$v "; PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 200 python3 tools/config3_run.py 1000000 5.0 5.0 | grep "config 3" || exit 1
  done
done
