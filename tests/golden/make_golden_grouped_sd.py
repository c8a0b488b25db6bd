#!/usr/bin/env python3
"""Reference fixtures for the standard deviations of the covariance parameters of grouped random effects
models with matrix_inversion_method = "cholesky" (GPB_GetCovPar(calc_std_dev = true) -> CalcStdDevCovPar
re_model_template.h:9775-9789 -> CalcFisherInformation_Only_Grouped_REs_Woodbury :9559-9651) from the
reference itself (oracle/_ref/ref_harness_grouped, mode=stddev):

    make -C oracle ref && python3 tests/golden/make_golden_grouped_sd.py
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from gpboost_amd import synthetic  # noqa: E402
from make_golden import fmt_pars, run_ref  # noqa: E402

OUT = os.path.join(HERE, "golden_grouped_sd.json")


def case(n, levels, cov_pars):
    g = synthetic.bench_groups(n, levels)
    y = synthetic.bench_grouped_y(g)
    r = run_ref(None, y, groups=g, cov_pars=fmt_pars(cov_pars), mode="stddev", matrix_inversion_method="cholesky")
    return dict(n=n, levels=list(levels), cov_pars=r["cov_pars"], std_dev=r["std_dev"])


def main():
    cases = {
        "sdg_k1_n5000": case(5000, (300,), (1.0, 0.5)),
        "sdg_k2_n20000": case(20000, (500, 50), (1.0, 1.0, 0.25)),
        "sdg_k3_n20000": case(20000, (400, 60, 7), (1.0, 1.0, 0.25, 0.1)),
        "sdg_k2_n3000_small": case(3000, (900, 3), (0.5, 2.0, 0.05)),
    }
    for k, v in cases.items():
        print(k, v["std_dev"], file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
