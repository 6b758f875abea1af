#!/bin/bash
# rocprofv3 kernel trace of the config-3 product path (run_fer_sweep --rng philox: one
# pscl_simulate call per SNR point), L = 8, 10^6 frames per point at the given SNRs.
#   bash tools/profile_sim_trace.sh <tag> [snr,snr,...]
set -o pipefail
tag=${1:-sim}; snrs=${2:-4.0,5.0}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/simtrace_${tag}
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o trace -- \
    python3 tools/sweep_timing.py 8 1000000 1048576 1 "$snrs" > "$out/timing.log" 2>&1 || { echo "trace failed"; tail -5 "$out/timing.log"; exit 1; }
python3 tools/sim_timeline.py "$out" > "$out/timeline.txt" 2>&1
cat "$out/timing.log"; head -60 "$out/timeline.txt"
