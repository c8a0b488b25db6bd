"""Per-application HBM-side bytes of the latent operator and VADU preconditioner from the raw
rocprofv3 --pmc CSVs of scripts/gpu_pmc_ops.sh. prof_op1.py ends with GPB_BenchLatentOperators(T, 20):
one warm-up operator + preconditioner application, then 20 operator applications (b_apply + bt_apply,
two dispatches each), then 20 preconditioner applications; so every dispatch after the last operator
dispatch belongs to the 20 timed preconditioner applications and the 40 operator dispatches before
them to the 20 timed operator applications. Counter values are KiB (x 1024). FETCH_SIZE is reported
raw and doubled (MI355X_MICROARCH.md §HBM: gfx950 tallies 128-B read requests at 64 B for wide
coalesced reads; the gathers here are 8 B per lane, outside that calibration).
Usage: pmc_ops_json.py DIR OUT.json"""
import csv
import glob
import json
import os
import sys

OPS = ("b_apply", "bt_apply")
d, out = sys.argv[1], sys.argv[2]


def short(k):
    return k.replace("gpb_amd::", "").replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (scripts/gpu_pmc_ops.sh, "
                  "scripts/pmc_ops_json.py), the 20 timed applications of GPB_BenchLatentOperators, eager launches",
       "unit": "bytes per application (KiB x 1024)", "columns": {}}
for T in (1, 51):
    entry = {}
    for P in ("FETCH_SIZE", "WRITE_SIZE"):
        paths = sorted(glob.glob(os.path.join(d, f"raw_t{T}_{P}", "**", "*counter_collection.csv"), recursive=True))
        if not paths:
            continue
        rows = {}
        with open(paths[0]) as f:
            for r in csv.DictReader(f):
                did = int(r["Dispatch_Id"])
                name = short(r["Kernel_Name"])
                v = rows.setdefault(did, [name, 0.])
                v[1] += float(r["Counter_Value"])
        ids = sorted(rows)
        last_op = max(i for i in ids if rows[i][0].startswith(OPS))
        pre = [i for i in ids if i > last_op]
        ops = [i for i in ids if i <= last_op and rows[i][0].startswith(OPS)][-40:]
        entry[P] = {"operator_KiB": sum(rows[i][1] for i in ops) / 20.,
                    "preconditioner_KiB": sum(rows[i][1] for i in pre) / 20.,
                    "operator_dispatches": len(ops), "preconditioner_dispatches": len(pre),
                    "operator_kernels": sorted({rows[i][0] for i in ops}),
                    "preconditioner_kernels": sorted({rows[i][0] for i in pre})}
    if "FETCH_SIZE" in entry and "WRITE_SIZE" in entry:
        f, w = entry["FETCH_SIZE"], entry["WRITE_SIZE"]
        for part in ("operator", "preconditioner"):
            entry[part + "_bytes_raw"] = (f[part + "_KiB"] + w[part + "_KiB"]) * 1024.
            entry[part + "_bytes"] = (2. * f[part + "_KiB"] + w[part + "_KiB"]) * 1024.
    res["columns"][str(T)] = entry
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
