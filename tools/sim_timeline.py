"""Per-SNR-point kernel timeline of a tools/profile_sim_trace.sh trace: kernels in start order with
their start offset and duration (us), grouped into points by the gaps between pscl_simulate
calls, and per-point totals by kernel.

    python tools/sim_timeline.py <trace dir>
"""
import collections
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "")))
rows.sort()
if not rows:
    sys.exit("no kernel trace")
# points: a channel_kernel launch starts each pscl_simulate chunk
points, cur = [], []
for r in rows:
    if "channel_kernel" in r[2] and cur:
        points.append(cur)
        cur = []
    cur.append(r)
points.append(cur)


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    return n[:70]


for i, pt in enumerate(points):
    t0, t1 = pt[0][0], max(r[1] for r in pt)
    print(f"== point {i}: {len(pt)} kernels, span {(t1 - t0) / 1e3:.1f} us")
    tot = collections.Counter()
    cnt = collections.Counter()
    for s, e, n, q in pt:
        tot[short(n)] += (e - s) / 1e3
        cnt[short(n)] += 1
    for n, t in tot.most_common():
        print(f"   {t:9.1f} us  x{cnt[n]:3d}  {n}")
    if i == len(points) - 1 or i < 3:
        for s, e, n, q in pt[:40]:
            print(f"      +{(s - t0) / 1e3:8.1f}  {(e - s) / 1e3:8.1f}  q{q}  {short(n)}")
