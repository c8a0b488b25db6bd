#!/usr/bin/env python3
"""Record the reference C API's GPB_* entry points (name, parameter count, header line) from
/root/reference/include/LightGBM/c_api.h into reference_c_api.json. Build container only; the JSON
is the fixture tests/test_capi.py checks the drop-in library against."""
import json
import os
import re

SRC = "/root/reference/include/LightGBM/c_api.h"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_c_api.json")


def main():
    txt = open(SRC).read()
    out = []
    for m in re.finditer(r"GPBOOST_C_EXPORT\s+int\s+(GPB_\w+)\s*\(([^;]*?)\)\s*;", txt, re.S):
        args = [a for a in m.group(2).split(",") if a.strip()]
        line = txt[: m.start()].count("\n") + 1
        out.append({"name": m.group(1), "nargs": len(args), "line": line})
    with open(OUT, "w") as f:
        json.dump({"source": "include/LightGBM/c_api.h", "functions": out}, f, indent=1)
    print(len(out), "functions")


if __name__ == "__main__":
    main()
