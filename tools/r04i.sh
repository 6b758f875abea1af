#!/bin/bash
# Round-4 GPU pass i: PMC of the config-3 product path at 5 dB (TX with the fused uncoded
# baseline, lane baseline decode, DL-SCL FS retry decodes and post passes) and of config 4.
set -o pipefail
bash tools/kernel_pmc.sh c3_5db python3 tools/config3_run.py 1000000 5.0 5.0 > gpurun_out/r04i_c3_pmc.txt 2>&1 || { tail -5 gpurun_out/r04i_c3_pmc.txt; exit 1; }
head -40 gpurun_out/r04i_c3_pmc.txt
bash tools/kernel_pmc.sh c4 python3 bench.py --list 4 --retries 8 --steps 2 --warmup 1 --no-cpu-baseline --extra none > gpurun_out/r04i_c4_pmc.txt 2>&1 || { tail -5 gpurun_out/r04i_c4_pmc.txt; exit 1; }
head -40 gpurun_out/r04i_c4_pmc.txt
