#!/usr/bin/env python3
"""Golden fixtures for GPB_OptimCovPar and GPB_GetCovPar(calc_std_dev) from the REFERENCE implementation.

Runs oracle/_ref/ref_harness in mode=fit (REModelTemplate::FindInitCovPar +
OptimLinRegrCoefCovPar with the Python package's default optimizer settings: "lbfgs",
lr_cov = -1, delta_rel_conv = -1, maxit = 1000) on portable synthetic inputs and writes
golden_fit.json next to this script. Build container only:

    make -C oracle ref && python3 tests/golden/make_golden_fit.py

Fixtures are data (inputs are regenerated from the LCG; outputs are reference results).
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, run_ref  # noqa: E402

sys.path.insert(0, ROOT)
from gpboost_amd import synthetic  # noqa: E402

# iterative-path settings for the latent cases: tight CG tolerance so the fit is deterministic
# up to summation order (the default 1e-2 is checked statistically elsewhere)
LATENT_ITER = dict(matrix_inversion_method="iterative", cg_delta_conv="1e-6", num_rand_vec_trace="50",
                   seed_rand_vec_trace="1")


def main():
    cases = {}
    coords, y = synthetic.rtest_gaussian_y(100)
    specs = {
        # R-package/tests/testthat/test_GPModel_gaussian_process.R:233-237: lbfgs estimate within 1e-2
        # (sum of absolute differences) of (0.03784221, 1.07390943, 0.11451432), nll 122.7771373
        "rtest_dense_exponential": dict(cov_fct="exponential", gp_approx="none"),
        "rtest_vecchia_m30_random": dict(cov_fct="exponential", gp_approx="vecchia", num_neighbors=30, ordering="random"),
        "rtest_dense_matern15_init": dict(cov_fct="matern", shape=1.5, gp_approx="none", init_cov_pars="0.1,1.6,0.2"),
    }
    for name, sp in specs.items():
        r = run_ref(coords, y, mode="fit", **sp)
        cases[name] = dict(data="rtest_gaussian", n=100, spec=sp, **{k: r[k] for k in r if k not in ("ok", "n", "d")})
        print(name, r["cov_pars"], r["nll"], r["num_it"], file=sys.stderr)

    n = 2000
    sc = synthetic.bench_coords(n)
    sy = synthetic.bench_gaussian_y(n)
    sspecs = {
        # n > 1000: the initial range comes from a 1000-point sample drawn with the model's RNG
        "synth2000_vecchia_m30_exp": dict(cov_fct="exponential", gp_approx="vecchia", num_neighbors=30, ordering="random"),
        "synth2000_vecchia_m20_gaussian": dict(cov_fct="gaussian", gp_approx="vecchia", num_neighbors=20, ordering="random"),
        "synth2000_vecchia_m30_matern25_init": dict(cov_fct="matern", shape=2.5, gp_approx="vecchia", num_neighbors=30,
                                                    ordering="random", init_cov_pars="0.2,0.8,0.05"),
        "synth2000_dense_exp": dict(cov_fct="exponential", gp_approx="none"),
    }
    for name, sp in sspecs.items():
        r = run_ref(sc, sy, mode="fit", **sp)
        cases[name] = dict(data="bench", n=n, spec=sp, **{k: r[k] for k in r if k not in ("ok", "n", "d")})
        print(name, r["cov_pars"], r["nll"], r["num_it"], file=sys.stderr)

    # latent models (Laplace + iterative methods), n = 500
    nl = 500
    lc = synthetic.bench_coords(nl)
    lspecs = {
        "latent500_bernoulli_m20": (synthetic.bench_bernoulli_y(lc),
                                    dict(cov_fct="exponential", gp_approx="vecchia", num_neighbors=20, ordering="random",
                                         likelihood="bernoulli_logit", **LATENT_ITER)),
        "latent500_gaussian_m20": (synthetic.bench_gaussian_y(nl),
                                   dict(cov_fct="exponential", gp_approx="vecchia_latent", num_neighbors=20,
                                        ordering="random", likelihood="gaussian", **LATENT_ITER)),
    }
    for name, (yy, sp) in lspecs.items():
        r = run_ref(lc, yy, mode="fit", **sp)
        cases[name] = dict(data="bench_latent", n=nl, spec=sp, **{k: r[k] for k in r if k not in ("ok", "n", "d")})
        print(name, r["cov_pars"], r.get("aux_pars"), r["nll"], r["num_it"], file=sys.stderr)

    # standard deviations (GPB_GetCovPar calc_std_dev = true; dense Gaussian), at fixed parameters.
    # rtest: R-package test_GPModel_gaussian_process.R cov_pars (estimate, std dev) pairs
    sd_cases = {
        "sd_rtest_exponential": (coords, y, dict(cov_fct="exponential", gp_approx="none"), "0.03784221,1.07390943,0.11451432"),
        "sd_rtest_matern15": (coords, y, dict(cov_fct="matern", shape=1.5, gp_approx="none"), "0.1,1.6,0.2"),
        "sd_rtest_matern25": (coords, y, dict(cov_fct="matern", shape=2.5, gp_approx="none"), "0.2,0.9,0.05"),
        "sd_rtest_gaussian": (coords, y, dict(cov_fct="gaussian", gp_approx="none"), "0.1,1.2,0.15"),
        "sd_synth2000_exponential": (sc, sy, dict(cov_fct="exponential", gp_approx="none"), "0.1,1.0,0.1"),
    }
    for name, (cx, yy, sp, pars) in sd_cases.items():
        r = run_ref(cx, yy, mode="stddev", cov_pars=pars, **sp)
        cases[name] = dict(data="rtest_gaussian" if cx is coords else "bench", n=cx.shape[0], spec=sp,
                           cov_pars=r["cov_pars"], std_dev=r["std_dev"])
        print(name, r["std_dev"], file=sys.stderr)

    with open(os.path.join(HERE, "golden_fit.json"), "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
