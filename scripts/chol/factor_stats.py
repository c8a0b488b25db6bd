"""Factor-phase breakdown of a rocprofv3 kernel trace of the Cholesky path: per kernel and, for the GEMM tiles, per
launch-size bucket (tiles per launch), totals over the trace's factorizations.
python scripts/chol/factor_stats.py <kernel_trace.csv>"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
phase = "other"
nfac = 0
by = collections.defaultdict(lambda: [0, 0.])
for r in rows:
    n = r["Kernel_Name"]
    if "chol_asm_tile" in n:
        if phase != "factor":
            nfac += 1
        phase = "factor"
    elif "chol_asmv" in n or "chol_fsolve1" in n or "chol_load_v" in n:
        phase = "solve"
    elif "chol_gather_s" in n:
        phase = "selinv"
    elif "chol_" not in n:
        phase = "other"
    if phase not in ("factor", "selinv"):
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    m = re.search(r"::(\w+)(?:<[^>]*>)?\(", n)
    short = phase + " " + (m.group(1) if m else n[:40])
    if "gemm" in short or "reduce" in short:
        g = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        b = 1
        while b < g:
            b *= 4
        short += f" tiles<={b}"
    by[short][0] += 1
    by[short][1] += d
print(f"factorizations: {nfac}")
tot = sum(v[1] for v in by.values())
print(f"factor + selinv kernels total {tot:.1f} ms")
for k, (c, t) in sorted(by.items(), key=lambda x: -x[1][1])[:30]:
    print(f"  {k:40s} {c:6d} launches {t:8.2f} ms {t / c * 1e3:8.1f} us avg")
