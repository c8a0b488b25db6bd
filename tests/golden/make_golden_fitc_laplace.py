#!/usr/bin/env python3
"""Reference fixtures for the FITC approximation with a Laplace likelihood (gp_approx = "fitc",
likelihood = "bernoulli_logit", matrix_inversion_method = "cholesky"), from the reference itself
(oracle/_ref/ref_harness): the approximate negative marginal log-likelihood and its gradient
(FindModePostRandEffCalcMLLFITC likelihoods.h:3090-3235, CalcGradNegMargLikelihoodLaplaceApproxFITC
:5397-5593), fits (GPB_OptimCovPar), predictions (PredictLaplaceApproxFITC :7157-7232) and the
gradient wrt the fixed effects (CalcGradientF). Build container only:

    make -C oracle ref && python3 tests/golden/make_golden_fitc_laplace.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, fmt_pars, run_ref  # noqa: E402

sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from gpboost_amd import synthetic  # noqa: E402

OUT = os.path.join(HERE, "golden_fitc_laplace.json")


def data(n):
    X = synthetic.bench_coords(n)
    y = synthetic.bench_bernoulli_y(X)
    return X, y


def spec_of(m, cov_fct="exponential", shape=0.5, sel="kmeans++", seed=0):
    return dict(cov_fct=cov_fct, shape=str(shape), gp_approx="fitc", num_ind_points=m, ind_points_selection=sel,
                seed=seed, likelihood="bernoulli_logit")


def case(n, m, cov_pars, **kw):
    X, y = data(n)
    spec = spec_of(m, **kw)
    r = run_ref(X, y, cov_pars=fmt_pars(cov_pars), mode="eval", **spec)
    return dict(n=n, m=m, cov_pars=list(cov_pars), spec=spec, nll=r["nll"], grad=r["grad"], ref_time_s=r["median_time"],
                ind_points=r["ind_points"])


def fit_case(n, m, **kw):
    X, y = data(n)
    spec = spec_of(m, **kw)
    r = run_ref(X, y, mode="fit", **spec)
    return dict(n=n, m=m, spec=spec, **{k: r[k] for k in r if k not in ("ok", "n", "d")})


def grad_f_case(n, m, cov_pars, **kw):
    X, y = data(n)
    fe = 0.3 * np.sin(3.0 * X[:, 0]) - 0.2
    spec = spec_of(m, **kw)
    r = run_ref(X, y, fe=fe, cov_pars=fmt_pars(cov_pars), mode="grad_f", **spec)
    ev = run_ref(X, y, fe=fe, cov_pars=fmt_pars(cov_pars), mode="eval", **spec)
    return dict(n=n, m=m, cov_pars=list(cov_pars), spec=spec, grad_f=r["grad_f"], nll=ev["nll"], grad=ev["grad"])


def pred_case(n, m, npred, cov_pars, cov=False, response=False, train_pts=0, **kw):
    X, y = data(n)
    Xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    if train_pts:
        Xp[:train_pts] = X[::max(1, n // train_pts)][:train_pts]
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([npred], dtype=np.int32).tobytes())
        f.write(np.asfortranarray(Xp).T.astype(np.float64).tobytes())
        ppath = f.name
    spec = spec_of(m, **kw)
    extra = {"predict_cov": "1"} if cov else {"predict_var": "1"}
    if response:
        extra["predict_response"] = "1"
    try:
        r = run_ref(X, y, cov_pars=fmt_pars(cov_pars), mode="predict", pred=ppath, **spec, **extra)
    finally:
        os.unlink(ppath)
    out = dict(n=n, m=m, npred=npred, cov_pars=list(cov_pars), spec=spec, response=response, train_pts=train_pts,
               mean=r["mean"])
    out["cov" if cov else "var"] = r["cov" if cov else "var"]
    return out


def main():
    cases = {
        "fl_exp_n2000_m100": case(2000, 100, (1.0, 0.1)),
        "fl_matern15_n3000_m80": case(3000, 80, (1.3, 0.15), cov_fct="matern", shape=1.5),
        "fl_gauss_n2500_m60_random": case(2500, 60, (0.8, 0.2), cov_fct="gaussian", shape=0.0, sel="random", seed=3),
        "fl_matern25_n4000_m300": case(4000, 300, (1.0, 0.1), cov_fct="matern", shape=2.5, seed=7),
        "fl_exp_n20000_m500": case(20000, 500, (1.0, 0.1)),
    }
    for k, v in cases.items():
        print(k, v["nll"], v["grad"], v["ref_time_s"], file=sys.stderr)
    fits = {
        "fit_fl_exp_n2000_m50": fit_case(2000, 50),
        "fit_fl_matern15_n3000_m100": fit_case(3000, 100, cov_fct="matern", shape=1.5),
    }
    for k, v in fits.items():
        print(k, v["cov_pars"], v["nll"], v["num_it"], file=sys.stderr)
    cases.update(fits)
    cases.update({
        "gradf_fl_exp_n2000_m80": grad_f_case(2000, 80, (1.0, 0.1)),
        "pred_fl_exp_var": pred_case(2000, 60, 300, (1.0, 0.1)),
        "pred_fl_exp_resp": pred_case(2000, 60, 300, (1.0, 0.1), response=True),
        "pred_fl_matern15_cov": pred_case(1500, 60, 100, (1.3, 0.15), cov_fct="matern", shape=1.5, cov=True),
        "pred_fl_train_pts_var": pred_case(2000, 50, 200, (1.0, 0.1), train_pts=60),
        "pred_fl_train_pts_cov": pred_case(2000, 50, 80, (1.0, 0.1), cov=True, train_pts=30),
    })
    with open(OUT, "w") as f:
        json.dump(cases, f)


if __name__ == "__main__":
    main()
