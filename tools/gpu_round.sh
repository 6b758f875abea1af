#!/bin/bash
# One GPU call: GPU tests, smoke, default bench, rocprofv3 kernel trace and PMC passes.
#   bash tools/gpu_round.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
  tail -3 gpurun_out/${tag}_gpu_tests.log
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/${tag}_smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${tag}_bench.log; exit 1; }
timeout -k 10 420 bash tools/profile_trace.sh ${tag} || { echo "trace failed"; exit 1; }
timeout -k 10 900 bash tools/profile_pmc.sh ${tag} || { echo "pmc failed"; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_${tag} 1000000 --json > gpurun_out/${tag}_pmc_summary.txt 2>&1
echo done
