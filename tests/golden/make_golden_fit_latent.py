#!/usr/bin/env python3
"""Reference fixtures for latent (Laplace / vecchia_latent) covariance fits at a tight CG tolerance
(GPB_OptimCovPar -> OptimLinRegrCoefCovPar, re_model_template.h:846-1700, with the iterative
Laplace-Vecchia objective likelihoods.h:2765-3076). At cg_delta_conv = 1e-8 the PCG solves are
converged far below the 1e-6 parity tolerance, so the fit path (iteration count, estimates) is
pinned by the algorithm rather than by rounding; the default-tolerance fits (make_golden_fit.py,
cg_delta_conv = 1e-6) stay as the looser cross-check. Build container only:

    make -C oracle ref && python3 tests/golden/make_golden_fit_latent.py
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, run_ref  # noqa: E402

sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from gpboost_amd import synthetic  # noqa: E402

TIGHT = dict(matrix_inversion_method="iterative", cg_delta_conv="1e-8", num_rand_vec_trace="50",
             seed_rand_vec_trace="1")


def offset(X):
    return 0.5 * np.sin(3 * X[:, 0]) - 0.3 * X[:, 1]


def main():
    cases = {}
    n = 2000
    X = synthetic.bench_coords(n)
    specs = {
        "latent2000_bernoulli_m30_tight": (synthetic.bench_bernoulli_y(X), None,
                                           dict(cov_fct="exponential", gp_approx="vecchia", num_neighbors=30,
                                                ordering="random", likelihood="bernoulli_logit", **TIGHT)),
        "latent2000_gaussian_m30_tight": (synthetic.bench_spatial_gaussian_y(X), None,
                                          dict(cov_fct="exponential", gp_approx="vecchia_latent", num_neighbors=30,
                                               ordering="random", likelihood="gaussian", **TIGHT)),
        "latent2000_bernoulli_offset_tight": (synthetic.bench_bernoulli_y(X), offset(X),
                                              dict(cov_fct="exponential", gp_approx="vecchia", num_neighbors=30,
                                                   ordering="random", likelihood="bernoulli_logit", **TIGHT)),
    }
    for name, (yy, fe, sp) in specs.items():
        r = run_ref(X, yy, fe=fe, mode="fit", **sp)
        cases[name] = dict(data="bench_latent", n=n, spec=sp, offset=fe is not None,
                           **{k: r[k] for k in r if k not in ("ok", "n", "d")})
        print(name, r["cov_pars"], r.get("aux_pars"), r["nll"], r["num_it"], file=sys.stderr)
    with open(os.path.join(HERE, "golden_fit_latent.json"), "w") as f:
        json.dump(cases, f)


if __name__ == "__main__":
    main()
