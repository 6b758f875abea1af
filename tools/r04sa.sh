#!/bin/bash
# Round-4 GPU pass sa: screen every retry chain (dl_screen=1) vs the default rule, final build.
set -o pipefail
for r in 1 2; do
  for t in "" "dl_screen=1"; do
    timeout -k 10 200 python3 tools/config3_run.py 1000000 5.0 5.0 $t | grep "config 3" || exit 1
    timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 6.5 $t | grep "config 3" || exit 1
  done
done
echo "config 4:"; timeout -k 10 300 bash tools/dl_tune.sh 2 - dl_screen=1 || exit 1
