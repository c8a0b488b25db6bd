"""Sum rocprofv3 --pmc counter values per kernel name (counter_collection CSV): per kernel the
dispatch count and the per-dispatch mean of every counter. Usage: pmc_by_kernel.py DIR OUT"""
import csv
import glob
import os
import sys
from collections import defaultdict

d, out = sys.argv[1], sys.argv[2]
path = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))[0]
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
with open(path) as f:
    for r in csv.DictReader(f):
        k = r["Kernel_Name"].replace("gpb_amd::", "").replace("(anonymous namespace)::", "").replace("void ", "")
        k = k.split("(")[0][:70]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
with open(out, "w") as f:
    for k in sorted(acc, key=lambda x: -sum(acc[x].values())):
        n = len(disp[k])
        vals = " ".join(f"{c}={v / n:.4g}" for c, v in sorted(acc[k].items()))
        hit, miss = acc[k].get("TCC_HIT_sum", 0.), acc[k].get("TCC_MISS_sum", 0.)
        rate = f" hit_rate={hit / (hit + miss):.3f}" if hit + miss > 0 else ""
        f.write(f"{n:8d} {k:70s} {vals}{rate}\n")
print(open(out).read())
