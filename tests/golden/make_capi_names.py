#!/usr/bin/env python3
"""Record the reference C API's GPB_* entry points (name, parameter count, parameter types, header
line) from /root/reference/include/LightGBM/c_api.h into reference_c_api.json. Build container only;
the JSON is the fixture tests/test_capi.py checks the drop-in library against. Parameter types are
normalised by param_type(), which tests/test_capi.py applies to include/gpboost_amd.h as well."""
import json
import os
import re

SRC = "/root/reference/include/LightGBM/c_api.h"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_c_api.json")


HANDLES = ("REModelHandle", "BoosterHandle", "DatasetHandle")   # typedef void* (c_api.h:29-31)


def param_type(decl: str) -> str:
    """'const double* init_cov_pars' -> 'const double*' (handles -> 'void*'; whitespace normalised)."""
    d = re.sub(r"\s+", " ", decl.replace("*", " * ")).strip()
    toks = d.split(" ")
    if len(toks) > 1 and re.match(r"^[A-Za-z_]\w*$", toks[-1]):
        toks = toks[:-1]   # drop the parameter name
    t = " ".join(toks).replace(" *", "*")
    for h in HANDLES:
        t = re.sub(r"\b%s\b" % h, "void*", t)
    return t


def main():
    txt = open(SRC).read()
    out = []
    for m in re.finditer(r"GPBOOST_C_EXPORT\s+int\s+(GPB_\w+)\s*\(([^;]*?)\)\s*;", txt, re.S):
        args = [a for a in m.group(2).split(",") if a.strip()]
        line = txt[: m.start()].count("\n") + 1
        out.append({"name": m.group(1), "nargs": len(args), "types": [param_type(a) for a in args], "line": line})
    with open(OUT, "w") as f:
        json.dump({"source": "include/LightGBM/c_api.h", "functions": out}, f, indent=1)
    print(len(out), "functions")


if __name__ == "__main__":
    main()
