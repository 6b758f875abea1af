#!/bin/bash
# Round-4 GPU pass o: config-3 sweep repeatability (8 back-to-back runs of tools/config3_run.py).
set -o pipefail
for r in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 python3 tools/config3_run.py 1000000 4.0 6.5 | grep "config 3" || exit 1
done
