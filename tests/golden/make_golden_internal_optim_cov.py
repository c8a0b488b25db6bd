#!/usr/bin/env python3
"""Golden fixtures for the internal covariance-parameter optimizers with linear regression covariates
(optimizer_coef "wls", the Gaussian default, re_model_template.h:1290-1549 with the GLS update :1327-1330) from the
REFERENCE implementation (oracle/_ref/ref_harness, mode=fit). Build container only:

    make -C oracle ref && python3 tests/golden/make_golden_internal_optim_cov.py

Fixtures are data (inputs regenerated from gpboost_amd.synthetic; outputs are reference results).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from gpboost_amd import synthetic  # noqa: E402
from make_golden import fmt_pars, run_ref  # noqa: E402

OUT = os.path.join(HERE, "golden_internal_optim_cov.json")


def data(name):
    if name == "rtest_linreg":   # test_GPModel_gaussian_process.R:432
        coords, y0 = synthetic.rtest_gaussian_y(100)
        Xc = synthetic.rtest_probit_X(100)
        return coords, Xc, y0 + Xc @ np.array([2., 2.])
    n = 2000
    coords = synthetic.bench_coords(n)
    Xc = np.column_stack([np.ones(n), np.sin(2 * np.pi * coords[:, 0])])
    return coords, Xc, synthetic.bench_gaussian_y(n) + Xc @ np.array([1., -0.5])


def main():
    cases = {}
    GD = dict(optimizer="gradient_descent", lr_cov="0.1", delta_rel_conv="1e-6")
    FS = dict(optimizer="fisher_scoring", lr_cov="1", delta_rel_conv="1e-6")
    specs = {
        "linreg_rtest_gd": ("rtest_linreg", dict(cov_fct="exponential", gp_approx="none", **GD)),
        "linreg_rtest_gd_crit_pars": ("rtest_linreg", dict(cov_fct="exponential", gp_approx="none",
                                                           convergence_criterion="relative_change_in_parameters", **GD)),
        "linreg_rtest_fisher": ("rtest_linreg", dict(cov_fct="exponential", gp_approx="none", **FS)),
        "linreg_synth2000_vecchia_gd": ("synth2000", dict(cov_fct="exponential", gp_approx="vecchia", num_neighbors=20,
                                                         ordering="random", **GD)),
    }
    for name, (dn, opts) in specs.items():
        coords, Xc, y = data(dn)
        r = run_ref(coords, y, X=Xc, mode="fit", **opts)
        cases[name] = dict(data=dn, spec=opts, **{k: r[k] for k in ("init_cov_pars", "cov_pars", "coef", "nll", "num_it")
                                                 if k in r})
        print(name, r.get("cov_pars"), r.get("coef"), r.get("nll"), r.get("num_it"), file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
