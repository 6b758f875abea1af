#!/bin/bash
# Round-4 GPU pass o: screening retry decodes (dl_screen) on the config-3 sweep and its points.
set -o pipefail
for r in 1 2; do
  for t in "" "dl_screen=1"; do
    timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 6.5 $t | grep "config 3" || exit 1
    timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 4.0 $t | grep "config 3" || exit 1
    timeout -k 10 200 python3 tools/config3_run.py 1000000 5.0 5.0 $t | grep "config 3" || exit 1
  done
done
