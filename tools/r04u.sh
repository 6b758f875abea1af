#!/bin/bash
# Round-4 GPU pass u: DL-SCL post-pass grid sized for fewer entry pairs per wavefront.
set -o pipefail
echo "config 4:"; timeout -k 10 400 bash tools/dl_tune.sh 2 - post_pairs=1 post_pairs=2 post_pairs=1,post_grid=4096 || exit 1
for r in 1 2; do
  for t in "" "post_pairs=1" "post_pairs=2"; do
    timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 6.5 $t | grep "config 3" || exit 1
    timeout -k 10 200 python3 tools/config3_run.py 1000000 5.0 5.0 $t | grep "config 3" || exit 1
  done
done
