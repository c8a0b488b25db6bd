"""Summarise a rocprofv3 kernel-trace CSV (too large to keep): per-kernel totals, the busy/idle
split of the traced span, the largest gaps and what preceded them. Usage: trace_summary.py DIR OUT"""
import csv
import glob
import os
import sys
from collections import defaultdict

d, out = sys.argv[1], sys.argv[2]
path = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
# the profiled (second) evaluation: everything after the largest host gap
gaps = [(rows[i + 1][0] - rows[i][1], i) for i in range(len(rows) - 1)]
cut = max(gaps)[1] + 1 if gaps else 0
ev = rows[cut:]
span = ev[-1][1] - ev[0][0]
busy = 0
last_end = ev[0][0]
tot = defaultdict(lambda: [0, 0])
gap_after = defaultdict(lambda: [0, 0])
for s, e, k in ev:
    busy += e - max(s, last_end) if e > last_end else 0
    last_end = max(last_end, e)
    name = k.replace("gpb_amd::", "").replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:80]
    tot[name][0] += 1
    tot[name][1] += e - s
for i in range(len(ev) - 1):
    g = ev[i + 1][0] - ev[i][1]
    if g > 0:
        n2 = ev[i + 1][2].replace("gpb_amd::", "").replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        gap_after[n2][0] += 1
        gap_after[n2][1] += g
with open(out, "w") as f:
    f.write(f"trace {path}: {len(rows)} kernels, evaluation = last {len(ev)} (cut at the largest gap)\n")
    f.write(f"span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms\n\n")
    f.write("kernel totals (count, total ms, avg us):\n")
    for k, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1]):
        f.write(f"  {c:8d} {t / 1e6:10.3f} {t / c / 1e3:9.2f}  {k}\n")
    f.write("\nidle time before kernels (count, total ms, avg us):\n")
    for k, (c, t) in sorted(gap_after.items(), key=lambda x: -x[1][1])[:25]:
        f.write(f"  {c:8d} {t / 1e6:10.3f} {t / c / 1e3:9.2f}  {k}\n")
print(open(out).read())
