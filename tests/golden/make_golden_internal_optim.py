#!/usr/bin/env python3
"""Golden fixtures for the reference's internal covariance-parameter optimizers ("gradient_descent" with
and without Nesterov acceleration, "fisher_scoring") from the REFERENCE implementation: oracle/_ref/ref_harness
and ref_harness_grouped in mode=fit with optimizer=... (REModelTemplate::OptimLinRegrCoefCovPar,
re_model_template.h:1290-1549). Build container only:

    make -C oracle ref && python3 tests/golden/make_golden_internal_optim.py

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

OUT = os.path.join(HERE, "golden_internal_optim.json")

GD = dict(optimizer="gradient_descent", lr_cov="0.1", delta_rel_conv="1e-6")
FS = dict(optimizer="fisher_scoring", lr_cov="1", delta_rel_conv="1e-6")


def _keep(r):
    return {k: r[k] for k in ("init_cov_pars", "cov_pars", "nll", "num_it") if k in r}


def main():
    cases = {}
    X, y = synthetic.rtest_gaussian_y(100)
    D = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    mean_dist = D[np.triu_indices(100, 1)].mean()
    init = fmt_pars([np.var(y, ddof=1) / 2, np.var(y, ddof=1) / 2, mean_dist / 3])
    # test_GPModel_gaussian_process.R:117-170 (init var(y)/2, var(y)/2, mean(dist)/3)
    rspecs = {
        "rtest_gd_nesterov": dict(GD),
        "rtest_gd_no_acc": dict(GD, use_nesterov_acc="0"),
        "rtest_gd_lr1": dict(GD, lr_cov="1"),
        "rtest_gd_crit_pars": dict(GD, convergence_criterion="relative_change_in_parameters"),
        "rtest_fisher": dict(FS),
        "rtest_gd_default": dict(optimizer="gradient_descent"),   # no init: FindInitCovPar, lr / delta defaults
        "rtest_fisher_default": dict(optimizer="fisher_scoring"),
    }
    for name, sp in rspecs.items():
        opts = dict(cov_fct="exponential", gp_approx="none", **sp)
        if name not in ("rtest_gd_default", "rtest_fisher_default"):
            opts["init_cov_pars"] = init
        r = run_ref(X, y, mode="fit", **opts)
        cases[name] = dict(data="rtest_gaussian", spec=opts, **_keep(r))
        print(name, r["cov_pars"], r["nll"], r["num_it"], file=sys.stderr)

    # dense and Vecchia, n = 2000 (synthetic bench data); Fisher scoring on the dense path only
    n = 2000
    sc = synthetic.bench_coords(n)
    sy = synthetic.bench_gaussian_y(n)
    sspecs = {
        "synth2000_dense_gd": dict(cov_fct="exponential", gp_approx="none", **GD),
        "synth2000_dense_fisher_matern15": dict(cov_fct="matern", shape=1.5, gp_approx="none", **FS),
        "synth2000_vecchia_gd": dict(cov_fct="exponential", gp_approx="vecchia", num_neighbors=20, ordering="random",
                                     **GD),
    }
    for name, opts in sspecs.items():
        r = run_ref(sc, sy, mode="fit", **opts)
        cases[name] = dict(data="bench", n=n, spec=opts, **_keep(r))
        print(name, r["cov_pars"], r["nll"], r["num_it"], file=sys.stderr)

    # grouped random effects (cholesky), K = 1 and K = 2
    for name, levels, opts in [
        ("grouped_k1_gd", (50,), dict(GD)),
        ("grouped_k1_fisher", (50,), dict(FS)),
        ("grouped_k2_gd", (80, 15), dict(GD)),
        ("grouped_k2_fisher", (80, 15), dict(FS)),
        ("grouped_k2_gd_no_acc_crit_pars", (80, 15),
         dict(GD, use_nesterov_acc="0", convergence_criterion="relative_change_in_parameters")),
    ]:
        ng = 3000
        g = synthetic.bench_groups(ng, levels)
        yg = synthetic.bench_grouped_y(g)
        opts = dict(matrix_inversion_method="cholesky", **opts)
        r = run_ref(None, yg, groups=g, mode="fit", **opts)
        cases[name] = dict(data="grouped", n=ng, levels=list(levels), spec=opts, **_keep(r))
        print(name, r["cov_pars"], r["nll"], r["num_it"], file=sys.stderr)

    # combined GP + grouped random effects (gp_approx = none), R-test data
    Xc, gc, yc = synthetic.rtest_combined_y(100)
    opts = dict(cov_fct="exponential", gp_approx="none", **GD)
    r = run_ref(Xc, yc, groups=gc.reshape(-1, 1), mode="fit", **opts)
    cases["combined_rtest_gd"] = dict(data="rtest_combined", spec=opts, **_keep(r))
    print("combined_rtest_gd", r["cov_pars"], r["nll"], r["num_it"], file=sys.stderr)

    # nelder_mead (OptimExternal -> OptimLib nm, optim_utils.h:642-643): default delta_rel_conv 1e-8
    NM = dict(optimizer="nelder_mead")
    for name, opts in {
        "nm_rtest_dense": dict(cov_fct="exponential", gp_approx="none", init_cov_pars=init, **NM),
        "nm_rtest_dense_default": dict(cov_fct="exponential", gp_approx="none", **NM),
        "nm_rtest_dense_crit_pars": dict(cov_fct="exponential", gp_approx="none", init_cov_pars=init,
                                         convergence_criterion="relative_change_in_parameters", delta_rel_conv="1e-6", **NM),
    }.items():
        r = run_ref(X, y, mode="fit", **opts)
        cases[name] = dict(data="rtest_gaussian", spec=opts, **_keep(r))
        print(name, r["cov_pars"], r["nll"], r["num_it"], file=sys.stderr)
    r = run_ref(sc, sy, mode="fit", cov_fct="matern", shape=1.5, gp_approx="vecchia", num_neighbors=20, ordering="random",
                **NM)
    cases["nm_synth2000_vecchia_matern15"] = dict(data="bench", n=n, spec=dict(cov_fct="matern", shape=1.5, gp_approx="vecchia",
                                                  num_neighbors=20, ordering="random", **NM), **_keep(r))
    g = synthetic.bench_groups(3000, (80, 15))
    r = run_ref(None, synthetic.bench_grouped_y(g), groups=g, mode="fit", matrix_inversion_method="cholesky", **NM)
    cases["nm_grouped_k2"] = dict(data="grouped", n=3000, levels=[80, 15],
                                  spec=dict(matrix_inversion_method="cholesky", **NM), **_keep(r))
    r = run_ref(Xc, yc, groups=gc.reshape(-1, 1), mode="fit", cov_fct="exponential", gp_approx="none", **NM)
    cases["nm_combined_rtest"] = dict(data="rtest_combined", spec=dict(cov_fct="exponential", gp_approx="none", **NM),
                                      **_keep(r))
    # Laplace models: dense (probit, R-test data) and FITC (poisson)
    from make_golden_latent_lik import data as lik_data
    Xp_, yp_ = lik_data("rtest_probit", 100)
    opts = dict(cov_fct="exponential", gp_approx="none", likelihood="bernoulli_probit", **NM)
    r = run_ref(Xp_, yp_, mode="fit", **opts)
    cases["nm_dense_probit_rtest"] = dict(data="lik", lik_data="rtest_probit", n=100, spec=opts, **_keep(r))
    Xq_, yq_ = lik_data("bench_pois", 1000)
    opts = dict(cov_fct="exponential", gp_approx="fitc", num_ind_points=50, likelihood="poisson", **NM)
    r = run_ref(Xq_, yq_, mode="fit", **opts)
    cases["nm_fitc_pois"] = dict(data="lik", lik_data="bench_pois", n=1000, spec=opts, **_keep(r))
    for k in ("nm_synth2000_vecchia_matern15", "nm_grouped_k2", "nm_combined_rtest", "nm_dense_probit_rtest", "nm_fitc_pois"):
        print(k, cases[k]["cov_pars"], cases[k]["nll"], cases[k]["num_it"], file=sys.stderr)

    with open(OUT, "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
