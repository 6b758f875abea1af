"""Host-side view of a rocprofv3 --kernel-trace --hip-trace run: HIP API calls longer than a
threshold (allocation, synchronisation, copies) in time order, beside the main-stream kernels.

    python tools/api_gaps.py <trace dir> [min_us]
"""
import csv
import glob
import sys

d = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
ev = []
for f in glob.glob(d + "/**/*hip_api_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if (e - s) / 1e3 >= min_us:
            ev.append((s, e, "API " + r["Function"]))
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if (e - s) / 1e3 >= min_us:
            ev.append((s, e, "K%s %s" % (r.get("Queue_Id", ""), r["Kernel_Name"][:60])))
ev.sort()
if not ev:
    sys.exit("no events")
t0 = ev[0][0]
tot = {}
for s, e, n in ev:
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  {n}")
    if n.startswith("API"):
        tot[n] = tot.get(n, 0.0) + (e - s) / 1e3
print("API totals (us, calls >= threshold):")
for n, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {v:10.1f}  {n}")

# busy host time: every HIP API call's duration summed by function, the blocking waits
# (hipEventSynchronize, hipStreamSynchronize, hipDeviceSynchronize) listed apart
calls = {}
for f in glob.glob(d + "/**/*hip_api_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        du = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c = calls.setdefault(r["Function"], [0, 0.0])
        c[0] += 1
        c[1] += du
wait = {k: v for k, v in calls.items() if "Synchronize" in k}
busy = {k: v for k, v in calls.items() if k not in wait}
print("API busy time (all calls, us):  total %.1f over %d calls" % (sum(v[1] for v in busy.values()),
                                                                      sum(v[0] for v in busy.values())))
for k, v in sorted(busy.items(), key=lambda x: -x[1][1])[:15]:
    print(f"  {v[1]:10.1f} {v[0]:7d}  {k}  ({v[1] / max(v[0], 1):.1f} us/call)")
print("API waits:")
for k, v in wait.items():
    print(f"  {v[1]:10.1f} {v[0]:7d}  {k}")

# per-call host busy time of pscl_dlscl_device calls: API time between consecutive
# hipEventSynchronize calls (one per pipelined call: the previous call's baseline), waits excluded
if len(sys.argv) > 3 and sys.argv[3] == "--per-call":
    rows = []
    for f in glob.glob(d + "/**/*hip_api_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
    rows.sort()
    cur, calls = None, []
    for s, e, fn in rows:
        if fn == "hipEventSynchronize":
            if cur:
                calls.append(cur)
            cur = {"busy": 0.0, "n": 0, "wait": (e - s) / 1e3, "t0": s}
        elif cur is not None and "Synchronize" not in fn:
            cur["busy"] += (e - s) / 1e3
            cur["n"] += 1
    for c in calls[-12:]:
        print(f"call: busy {c['busy']:8.1f} us over {c['n']:4d} API calls, then waited {c['wait']:8.1f} us")
