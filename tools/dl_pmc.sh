#!/bin/bash
# rocprofv3 PMC passes on the DL-SCL bench (config 4), summarised per kernel (name filter).
#   bash tools/dl_pmc.sh <tag> <kernel-substring> [lib variant]
set -o pipefail
tag=$1; kname=${2:-dl_post}; v=$3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/dlpmc_${tag}
mkdir -p "$out"
lp=""; [ -n "$v" ] && lp=tools/_variant/lib_$v.so
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT" "SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  PSCL_LIB_PATH=$lp timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o pmc -- \
      python3 bench.py --list 4 --retries 8 --steps 2 --warmup 1 --no-cpu-baseline --extra none > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -3 "$out/p$i.log"; exit 1; }
done
python3 - "$out" "$kname" <<'PY'
import collections, csv, glob, sys
agg = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    print(f"{k:24s} mean {sum(v)/len(v):.5g}  max {max(v):.5g}  n {len(v)}")
PY
