#!/usr/bin/env python3
"""Reference fixtures for linear regression covariates (GPB_OptimLinRegrCoefCovPar / GPB_GetCoef)
and for the training-data random-effect predictions (GPB_PredictREModelTrainingDataRandomEffects).
Build container only (about a minute on 8 cores):

    make -C oracle ref && python3 tests/golden/make_golden_cov.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, run_ref  # noqa: E402

sys.path.insert(0, ROOT)
from gpboost_amd import synthetic  # noqa: E402


def main():
    out = {}
    # ---- fits with covariates (default optimizer: lbfgs + wls, nugget profiled out)
    for name, n, spec in [("vecchia_fit_X", 2000, dict(gp_approx="vecchia", num_neighbors=30, ordering="random")),
                          ("dense_fit_X", 500, dict(gp_approx="none")),
                          ("vecchia_fit_X_matern15", 1500, dict(gp_approx="vecchia", num_neighbors=20,
                                                                ordering="random", cov_fct="matern", shape=1.5))]:
        X = synthetic.bench_coords(n)
        Xc = synthetic.bench_covariates(n, 2)
        y = synthetic.bench_gaussian_y_cov(X, Xc)
        sp = dict(cov_fct="exponential")
        sp.update(spec)
        r = run_ref(X, y, X=Xc, mode="fit", **sp)
        out[name] = dict(n=n, p=Xc.shape[1], spec=sp, cov_pars=r["cov_pars"], coef=r["coef"],
                         coef_std_dev=r["coef_std_dev"], init_cov_pars=r["init_cov_pars"], num_it=r["num_it"],
                         nll=r["nll"], cov_pars_std_dev=r.get("cov_pars_std_dev"))
        print(name, r["cov_pars"], r["coef"], r["num_it"], file=sys.stderr)
    # ---- training-data random effects (Gaussian: mean and variance; bernoulli: the mode)
    for name, n, spec in [("vecchia_pred_train", 2000, dict(gp_approx="vecchia", num_neighbors=30, ordering="random")),
                          ("dense_pred_train", 500, dict(gp_approx="none"))]:
        X = synthetic.bench_coords(n)
        y = synthetic.bench_gaussian_y(n)
        r = run_ref(X, y, mode="pred_train", cov_fct="exponential", cov_pars="0.1,1.0,0.1", **spec)
        out[name] = dict(n=n, spec=spec, cov_pars=[0.1, 1.0, 0.1], mean=r["mean"], var=r["var"])
        print(name, r["mean"][:3], r["var"][:3], file=sys.stderr)
    n = 2000
    X = synthetic.bench_coords(n)
    yb = synthetic.bench_bernoulli_y(X)
    r = run_ref(X, yb, mode="pred_train", cov_fct="exponential", gp_approx="vecchia", likelihood="bernoulli_logit",
                matrix_inversion_method="iterative", num_neighbors=30, ordering="random", cov_pars="1.0,0.1",
                cg_delta_conv="1e-10", num_rand_vec_trace="50", seed_rand_vec_trace="1")
    out["bernoulli_pred_train"] = dict(n=n, cov_pars=[1.0, 0.1], cg_delta_conv=1e-10, mean=r["mean"])
    print("bernoulli_pred_train", r["mean"][:3], file=sys.stderr)
    with open(os.path.join(HERE, "golden_cov.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
