#!/bin/bash
# Wall time of BASELINE config 5 through the CLI: run_ber_sweep --rng philox, NR polar E=256,
# K = 64 + CRC-24, L = 8, 4..6 dB, the reference's default caps; per --batch value.
#   bash tools/ber_timing.sh "<batch values>"   ("default" = the CLI default)
set -o pipefail
mkdir -p gpurun_out/ber
for b in $1; do
  extra=""; [ "$b" != default ] && extra="--batch $b"
  t0=$(date +%s.%N)
  timeout -k 10 300 python -m polar_code_amd.eval.run_ber_sweep --scheme nr_polar_scl --K_payload 64 --K_crc 24 --E 256 \
      --M 8 --EbN0_lo 4 --EbN0_hi 6 --EbN0_step 1 --rng philox $extra --out gpurun_out/ber/$b.csv > gpurun_out/ber/$b.log 2>&1 || { echo "$b failed"; tail -5 gpurun_out/ber/$b.log; exit 1; }
  t1=$(date +%s.%N)
  echo "batch=$b wall $(python3 -c "print(round($t1-$t0,2))") s"; tail -3 gpurun_out/ber/$b.csv
done
