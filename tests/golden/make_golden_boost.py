#!/usr/bin/env python3
"""Reference fixtures for the GPBoost algorithm's covariance update: three
consecutive boosting rounds of REModel::OptimCovPar(..., called_in_GPBoost_algorithm = true,
reuse_learning_rates_gp_model) followed by REModel::CalcGradient(..., calc_cov_factor = false), as
the boosting objective runs them (regression_objective.hpp:153-182), on scores F_r = scale_r * F.
Produced by the reference itself (oracle/_ref/ref_harness, mode=boost). Build container only:

    make -C oracle ref && python3 tests/golden/make_golden_boost.py
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

SCALES = [0.5, 1.0, 1.5]


def score(X):
    """A boosting-score-like F(x) (the same offset as make_golden_lagaboost.py)."""
    return 0.5 * np.sin(3 * X[:, 0]) - 0.3 * X[:, 1]


def main():
    out = {"scales": SCALES}
    sc = ",".join(repr(s) for s in SCALES)
    # Gaussian, exact Vecchia and dense: y_r = F_r - label, the nugget profiled out
    for name, n, spec in [("gauss_vecchia", 2000, dict(gp_approx="vecchia", num_neighbors=30, ordering="random")),
                          ("gauss_dense", 500, dict(gp_approx="none"))]:
        X = synthetic.bench_coords(n)
        y = synthetic.bench_gaussian_y(n)
        for reuse in (1, 0):
            r = run_ref(X, y, fe=score(X), mode="boost", cov_fct="exponential", scales=sc, reuse=str(reuse), **spec)
            key = f"{name}_reuse{reuse}"
            out[key] = dict(n=n, spec=spec, reuse=reuse, rounds=r["rounds"])
            print(key, [(rr["cov_pars"], rr["num_it"]) for rr in r["rounds"]], file=sys.stderr)
    # bernoulli_logit Laplace + Vecchia, iterative: tight CG tolerance (parity to 1e-6) and the default
    n = 1000
    X = synthetic.bench_coords(n)
    yb = synthetic.bench_bernoulli_y(X)
    lat = dict(cov_fct="exponential", gp_approx="vecchia", likelihood="bernoulli_logit",
               matrix_inversion_method="iterative", num_neighbors=30, ordering="random",
               num_rand_vec_trace="50", seed_rand_vec_trace="1")
    for cg in ("1e-8",):
        r = run_ref(X, yb, fe=score(X), mode="boost", scales=sc, reuse="1", cg_delta_conv=cg, **lat)
        key = f"bernoulli_cg{cg}"
        out[key] = dict(n=n, cg_delta_conv=float(cg), reuse=1, rounds=r["rounds"])
        print(key, [(rr["cov_pars"], rr["num_it"]) for rr in r["rounds"]], file=sys.stderr)
    with open(os.path.join(HERE, "golden_boost.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
