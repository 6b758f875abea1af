#!/bin/bash
# Round-4 GPU pass w: lane kernel LDS frame padding (bank mapping of the 4 frames of a b128 lane group).
set -o pipefail
bash tools/ab_bench.sh "prod fp8 fp24" 3 || exit 1
for v in prod fp8 fp24; do
  PSCL_LIB_PATH=tools/_variant/lib_$v.so bash tools/kernel_pmc.sh w_$v python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --extra none > gpurun_out/r04w_$v.txt 2>&1 || { tail -5 gpurun_out/r04w_$v.txt; exit 1; }
  echo "$v: $(grep -A1 'scl_lane_kernel<8, 1, false>' gpurun_out/r04w_$v.txt | tail -1 | cut -c1-400)"
done
