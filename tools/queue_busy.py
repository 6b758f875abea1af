"""Queue occupancy of a rocprofv3 kernel trace: per queue the busy time and the idle gaps between its
kernels, and the time no kernel runs at all, over the window from the first kernel whose name
contains `start` (default: the last channel_kernel-led sweep's first baseline) to the end.

    python tools/queue_busy.py <trace dir> [first-kernel substring] [occurrence]
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
key = sys.argv[2] if len(sys.argv) > 2 else "channel_kernel"
occ = int(sys.argv[3]) if len(sys.argv) > 3 else 0
hits = [i for i, r in enumerate(rows) if key in r[2]]
i0 = hits[occ]
win = rows[i0:]
t0, t1 = win[0][0], max(r[1] for r in win)
print(f"window {(t1 - t0) / 1e3:.1f} us from {key} #{occ}, {len(win)} kernels")
byq = collections.defaultdict(list)
for s, e, n, q in win:
    byq[q].append((s, e, n))
for q, ks in sorted(byq.items()):
    busy = sum(e - s for s, e, _ in ks) / 1e3
    gaps = [(ks[i + 1][0] - ks[i][1]) / 1e3 for i in range(len(ks) - 1)]
    big = sorted(((g, ks[i][2][:40], ks[i + 1][2][:40]) for i, g in enumerate(gaps)), reverse=True)[:4]
    print(f"queue {q}: {len(ks)} kernels, busy {busy:.1f} us, idle gaps total {sum(g for g in gaps if g > 0):.1f} us; largest:")
    for g, a, b in big:
        print(f"     {g:8.1f} us  after {a} -> {b}")
# time with no kernel running
ev = sorted([(s, 1) for s, e, _, _ in win] + [(e, -1) for s, e, _, _ in win])
depth, last, idle = 0, t0, 0
for t, d in ev:
    if depth == 0 and t > last:
        idle += t - last
    depth += d
    last = t
print(f"no kernel running: {idle / 1e3:.1f} us of {(t1 - t0) / 1e3:.1f}")
