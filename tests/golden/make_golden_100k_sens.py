#!/usr/bin/env python3
"""Rounding sensitivity of the REFERENCE's config-5 evaluation at the default cg_delta_conv = 1e-2
(bernoulli_logit Laplace + Vecchia m = 30, n = 100k): the same evaluation at covariance parameters
perturbed by a few ulps (relative 1e-14). Its thread-count spread is zero in the gradient
(make_golden_100k_tight.py), so this is the reference's own measure of how far two correct
implementations that round differently can land apart at the default tolerance. Appends
"bernoulli_sensitivity" to golden_100k.json. Build container only (~4 CPU-minutes):

    make -C oracle ref && python3 tests/golden/make_golden_100k_sens.py
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


def main():
    path = os.path.join(HERE, "golden_100k.json")
    with open(path) as f:
        out = json.load(f)
    n = 100_000
    X = synthetic.bench_coords(n)
    yb = synthetic.bench_bernoulli_y(X)
    spec = dict(mode="eval", cov_fct="exponential", gp_approx="vecchia", likelihood="bernoulli_logit",
                matrix_inversion_method="iterative", num_neighbors=30, ordering="random",
                num_rand_vec_trace="50", seed_rand_vec_trace="1", cg_delta_conv="1e-2")
    runs = []
    for pars in ([1.0 * (1 + 1e-14), 0.1], [1.0 * (1 - 1e-14), 0.1], [1.0, 0.1 * (1 + 1e-14)],
                 [1.0, 0.1 * (1 - 1e-14)]):
        r = run_ref(X, yb, cov_pars=",".join(repr(v) for v in pars), **spec)
        runs.append(dict(cov_pars=pars, nll=r["nll"], grad=r["grad"]))
        print(pars, r["nll"], r["grad"], file=sys.stderr, flush=True)
    out["bernoulli_sensitivity"] = dict(n=n, rel_perturbation=1e-14, cg_delta_conv=1e-2, runs=runs)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
