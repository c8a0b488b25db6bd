"""Busy time vs wall time of a rocprofv3 kernel trace, per segment split at idle gaps > 5 ms, and the per-kernel
totals of the last segment. Usage: trace_gaps.py DIR"""
import collections
import csv
import glob
import os
import sys

path = sorted(glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True))[0]
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        nm = r["Kernel_Name"].replace("gpb_amd::", "").replace("(anonymous namespace)::", "").split("(")[0]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm.replace("void ", "")[:48],
                     int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
rows.sort()
segs, st, prev = [], 0, rows[0][1]
for i, (s, e, n, g) in enumerate(rows):
    if s - prev > 5e6:
        segs.append((st, i))
        st = i
    prev = max(prev, e)
segs.append((st, len(rows)))
for a, b in segs:
    R = rows[a:b]
    wall = (max(r[1] for r in R) - R[0][0]) / 1e6
    busy = sum(r[1] - r[0] for r in R) / 1e6
    print(f"segment: {b - a} launches, wall {wall:.2f} ms, busy {busy:.2f} ms")
a, b = segs[-1]
by = collections.defaultdict(lambda: [0, 0.])
for s, e, n, g in rows[a:b]:
    by[n][0] += 1
    by[n][1] += (e - s) / 1e6
for n, (c, t) in sorted(by.items(), key=lambda x: -x[1][1])[:14]:
    print(f"  {n:48s} {c:6d} {t:9.2f} ms {t / c * 1e3:8.1f} us")
