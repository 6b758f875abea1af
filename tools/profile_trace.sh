#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench (run on the GPU box from the repo root).
#   bash tools/profile_trace.sh <tag> [bench args...]
set -o pipefail
tag=${1:-r01}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_${tag}
mkdir -p "$out"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o trace -- \
    python3 bench.py --steps 20 --warmup 1 --no-cpu-baseline --extra none "$@" > "$out/bench.log" 2>&1
