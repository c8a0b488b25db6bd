"""Attribute the kernels of a rocprofv3 kernel trace of the Cholesky path to its phases (factor / solve /
selected inverse / other) by the phase-opening kernels. python scripts/chol/phase_stats.py <kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
phase = "other"
acc, cnt = collections.defaultdict(float), collections.Counter()
for r in rows:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    if "chol_asm_tile" in n:
        phase = "factor"
    elif "chol_asmv" in n:
        phase = "solve"
    elif "chol_gather_s" in n:
        phase = "selinv"
    elif "chol_" not in n:
        phase = "other"
    short = n.split("(anonymous namespace)::")[-1].split("(")[0]
    acc[(phase, short)] += d
    cnt[(phase, short)] += 1
tot = collections.defaultdict(float)
for (ph, _), v in acc.items():
    tot[ph] += v
print({k: round(v, 1) for k, v in tot.items()})
for k, v in sorted(acc.items(), key=lambda x: -x[1])[:25]:
    print(k, cnt[k], "%.1f ms" % v, "%.1f us avg" % (1e3 * v / cnt[k]))
