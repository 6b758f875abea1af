#!/bin/bash
# rocprofv3 kernel + HIP API trace of the pipelined DL-SCL bench (config 4), to see where the host
# waits between a call's baseline and the next call's launches.   bash tools/profile_dl_api.sh <tag>
set -o pipefail
tag=${1:-p4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_dlapi_${tag}
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d "$out" -o trace -- \
    python3 bench.py --list 4 --retries 8 --steps 4 --warmup 1 --no-cpu-baseline --extra none > "$out/bench.log" 2>&1
ls "$out"
