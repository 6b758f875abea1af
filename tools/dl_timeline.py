"""Kernel timeline of a DL-SCL bench trace (tools/profile_dl_trace.sh): every kernel in start order
with its queue, start offset from the first baseline decode of the window and duration (us), for a
window of consecutive steps in the middle of the timed region.

    python tools/dl_timeline.py <trace dir> [first step] [steps]   (steps 0: to the trace's end)
"""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "")))
rows.sort()
first = int(sys.argv[2]) if len(sys.argv) > 2 else 3
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 2


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:48]


base = [r for r in rows if "scl_lane_kernel<4, 1, false" in r[2] or "scl_lane_kernel<8, 1, false" in r[2]]
if len(base) < first + max(nsteps, 1) + (nsteps > 0):
    sys.exit(f"only {len(base)} baseline decodes")
# steps 0: from baseline decode `first` to the end of the trace (a standalone sweep point)
t0, t1 = base[first][0], base[first + nsteps][0] if nsteps else max(r[1] for r in rows)
nsteps = max(nsteps, 1)
print(f"window: baseline decodes {first}..{first + nsteps - 1}, {(t1 - t0) / 1e3:.1f} us "
      f"({(t1 - t0) / 1e3 / nsteps:.1f} us per step)")
busy = {}
for s, e, n, q in rows:
    if e < t0 or s > t1:
        continue
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3}  {short(n)}")
    k = short(n)
    busy[k] = busy.get(k, 0.0) + (min(e, t1) - max(s, t0)) / 1e3
print("kernel-time in the window by kernel (us, overlapping):")
for k, v in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"  {v:9.1f}  {k}")
