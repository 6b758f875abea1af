#!/bin/bash
# Post-pass cost by ablation (timing only, results invalid in the variants): per library variant,
# rocprofv3 kernel stats of the config-3 5 dB point and of config 4; prints the dl_post_kernel total
# and each run's wall line.   bash tools/post_ablate.sh <tag> "<variant names>"  (product = "prod")
set -o pipefail
tag=$1; vars=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$tag; mkdir -p $out
for v in $vars; do
  lib=""; [ "$v" != "prod" ] && lib=tools/_variant/lib_$v.so
  for w in c3 c4; do
    if [ $w = c3 ]; then cmd="python3 tools/config3_run.py 1000000 5 5"; else cmd="python3 bench.py --list 4 --retries 8 --steps 6 --warmup 2 --no-cpu-baseline --extra none"; fi
    PSCL_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${v}_$w -o t -- $cmd > $out/${v}_$w.log 2>&1 || { echo "$v $w failed"; tail -5 $out/${v}_$w.log; exit 1; }
    post=$(python3 -c "
import csv,glob
t=0;n=0
for f in glob.glob('$out/${v}_$w/*kernel_stats.csv'):
  for r in csv.DictReader(open(f)):
    if 'dl_post_kernel' in r['Name']: t+=float(r['TotalDurationNs']); n+=int(r['Calls'])
print(round(t/1e3,1),'us in',n,'posts')")
    wall=$(python3 -c "
import json
for l in open('$out/${v}_$w.log'):
  if l.startswith('{'): print('ms/step', round(json.loads(l)['ms_per_step'],3))
  elif 'frames/s' in l: print(l.strip()[-60:])" | tail -1)
    echo "$v $w post $post | $wall"
  done
done
