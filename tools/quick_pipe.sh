set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fer.py tests/test_gpu_screening.py -x -q --timeout 200 --timeout-method thread -k "pipelined or split_chains or device_retry" > gpurun_out/p2_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/p2_tests.log; exit 1; }
tail -2 gpurun_out/p2_tests.log
timeout -k 10 300 python bench.py > gpurun_out/p2_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/p2_bench.log; exit 1; }
python -c "
import json; d=json.loads([l for l in open('gpurun_out/p2_bench.log') if l.startswith('{')][-1])
print('value', round(d['value']/1e6,1), 'ms', round(d['ms_per_step'],3), 'launch', round(d['roofline']['avg_launch_ms'],3), 'parity', d['parity']['mismatches'])
for k,v in (d['extra_configs'] or {}).items(): print(k, round(v['value']/1e6,1), round(v.get('ms_per_step') or 0,3), (v.get('parity') or {}).get('mismatches'), v.get('dl_scl'))
"
