"""Summarise rocprofv3 CSV output per kernel (runs on the GPU box; raw CSVs are large).

usage: pmc_summarize.py <rocprof dir> <out.csv>
  kernel traces  -> kernel, calls, mean_us, total_ms
  counter passes -> kernel, calls, <counter>_mean (per dispatch) for every counter
"""
import collections
import csv
import glob
import os
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("gpb_amd::", "")
    return name.split("(")[0][:90]


def main(d, out):
    rows = []
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if tr:
        acc = collections.defaultdict(list)
        for f in tr:
            for r in csv.DictReader(open(f)):
                acc[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
            rows.append({"kernel": k, "calls": len(v), "mean_us": sum(v) / len(v), "total_ms": sum(v) / 1e3})
    if cc:
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for f in cc:
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
        for k, cs in acc.items():
            n = len(disp[k])
            row = {"kernel": k, "calls": n}
            for c, v in cs.items():
                row[c + "_mean"] = v / n
            rows.append(row)
    keys = []
    for r in rows:
        for k in r:
            if k not in keys:
                keys.append(k)
    with open(out, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=keys)
        w.writeheader()
        for r in rows:
            w.writerow(r)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
