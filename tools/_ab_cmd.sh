set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_baseline_configs.py tests/test_gpu_fer.py tests/test_dl_ties.py > gpurun_out/r06z_t.log 2>&1 || { tail -30 gpurun_out/r06z_t.log; exit 1; }
tail -1 gpurun_out/r06z_t.log
timeout -k 10 400 bash tools/ab_bench.sh "prod pk4" 3 --list 4 --retries 8 || exit 1
for r in 1 2 3; do for v in prod pk4; do
  PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 120 python3 tools/config3_run.py 1000000 5.0 5.0 | sed "s/^/$v /" || exit 1
done; done
for r in 1 2; do for v in prod pk4; do
  PSCL_LIB_PATH=tools/_variant/lib_$v.so timeout -k 10 120 python3 tools/config3_run.py 1000000 4.0 6.5 | sed "s/^/$v /" || exit 1
done; done
