#!/bin/bash
# Round-4 GPU pass l: DL-SCL knob sweep (config 4) and the N = 1024 occupancy A/B.
set -o pipefail
timeout -k 10 700 bash tools/dl_tune.sh 2 - dl_split=1 post_grid=1024 post_grid=4096 post_grid=256 retry_wpg=2 side_priority=1 || exit 1
for v in prod l1024w1; do echo "long ($v):"; PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 300 python3 tools/long_bench.py 2>&1 | grep "N=1024 K=512 L=8" || exit 1; done
echo "history instances with aggregated counters (diagnostic variant):"
PSCL_LIB_PATH=tools/_variant/lib_histagg.so timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -q --timeout 120 2>&1 | grep -E "passed|failed|FAILED" | head -20
