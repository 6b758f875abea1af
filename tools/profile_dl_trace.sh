#!/bin/bash
# rocprofv3 kernel-trace summary of the DL-SCL bench (config 4: L=4, 8 flips, beta_M4), per-kernel
# times of the baseline decode and the retry rounds.   bash tools/profile_dl_trace.sh <tag>
set -o pipefail
tag=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_dl_${tag}
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o trace -- \
    python3 bench.py --list 4 --retries 8 --steps 5 --warmup 1 --no-cpu-baseline --extra none > "$out/bench.log" 2>&1
