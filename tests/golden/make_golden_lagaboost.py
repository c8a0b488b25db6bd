#!/usr/bin/env python3
"""Reference fixtures for the GPBoost-algorithm entry points: likelihood
evaluations with fixed effects F (the boosting score, an offset of the location parameter), the
gradient wrt F (REModel::CalcGradient -> CalcGradientF, re_model_template.h:3021-3043) and a fit
with an offset (REModel::OptimCovPar(nullptr, score), regression_objective.hpp:178). Build container
only (about a minute on 8 cores):

    make -C oracle ref && python3 tests/golden/make_golden_lagaboost.py
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


def offset(X):
    """A smooth boosting-score-like fixed effect F(x)."""
    return 0.5 * np.sin(3 * X[:, 0]) - 0.3 * X[:, 1]


def main():
    out = {}
    it = dict(cg_delta_conv="1e-10", num_rand_vec_trace="50", seed_rand_vec_trace="1")
    n = 2000
    X = synthetic.bench_coords(n)
    F = offset(X)
    yb = synthetic.bench_bernoulli_y(X)
    lat = dict(cov_fct="exponential", gp_approx="vecchia", likelihood="bernoulli_logit",
               matrix_inversion_method="iterative", num_neighbors=30, ordering="random")
    ev = run_ref(X, yb, fe=F, mode="eval", cov_pars="1.0,0.1", **lat, **it)
    gf = run_ref(X, yb, fe=F, mode="grad_f", cov_pars="1.0,0.1", **lat, **it)
    out["bernoulli_offset"] = dict(n=n, cov_pars=[1.0, 0.1], cg_delta_conv=1e-10, nll=ev["nll"], grad=ev["grad"],
                                   grad_f=gf["grad_f"])
    print("bernoulli_offset", ev["nll"], ev["grad"], gf["grad_f"][:3], file=sys.stderr)
    fit = run_ref(X, yb, fe=F, mode="fit", **lat, cg_delta_conv="1e-6", num_rand_vec_trace="50",
                  seed_rand_vec_trace="1")
    out["bernoulli_offset_fit"] = dict(n=n, cg_delta_conv=1e-6, cov_pars=fit["cov_pars"], nll=fit["nll"],
                                       num_it=fit["num_it"], init_cov_pars=fit["init_cov_pars"])
    print("bernoulli_offset_fit", fit["cov_pars"], fit["num_it"], file=sys.stderr)
    # vecchia_latent Gaussian with an offset (aux = error variance 0.1)
    yg = synthetic.bench_gaussian_y(n) + F
    lg = dict(cov_fct="exponential", gp_approx="vecchia_latent", likelihood="gaussian",
              matrix_inversion_method="iterative", num_neighbors=30, ordering="random")
    ev = run_ref(X, yg, fe=F, mode="eval", cov_pars="1.0,0.1", aux_pars="0.1", **lg, **it)
    gf = run_ref(X, yg, fe=F, mode="grad_f", cov_pars="1.0,0.1", aux_pars="0.1", **lg, **it)
    out["gauss_latent_offset"] = dict(n=n, cov_pars=[1.0, 0.1], aux=0.1, cg_delta_conv=1e-10, nll=ev["nll"],
                                      grad=ev["grad"], grad_f=gf["grad_f"])
    print("gauss_latent_offset", ev["nll"], ev["grad"], file=sys.stderr)
    # Gaussian (exact): gradient wrt F = Psi^-1 (F - y) / sigma^2 (the input is the residual)
    for name, nn, spec in [("vecchia_grad_f", 2000, dict(gp_approx="vecchia", num_neighbors=30, ordering="random")),
                           ("dense_grad_f", 500, dict(gp_approx="none"))]:
        Xn = synthetic.bench_coords(nn)
        r = offset(Xn) - synthetic.bench_gaussian_y(nn)
        gf = run_ref(Xn, r, mode="grad_f", cov_fct="exponential", cov_pars="0.1,1.0,0.1", **spec)
        out[name] = dict(n=nn, spec=spec, cov_pars=[0.1, 1.0, 0.1], grad_f=gf["grad_f"])
        print(name, gf["grad_f"][:3], file=sys.stderr)
    with open(os.path.join(HERE, "golden_lagaboost.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
