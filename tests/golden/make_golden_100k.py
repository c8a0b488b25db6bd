#!/usr/bin/env python3
"""Reference values at the BASELINE size (n = 100k, m = 30, bench data) for the GPU parity tests:
the exact Gaussian Vecchia L-BFGS unit (config 3a), the latent PCG + SLQ evaluation at the
default tolerance (config 3b) and the bernoulli_logit Laplace evaluation (config 5). Build container only (about two minutes on 8 cores):

    make -C oracle ref && python3 tests/golden/make_golden_100k.py
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
    n = 100_000
    X = synthetic.bench_coords(n)
    y = synthetic.bench_gaussian_y(n)
    ex = run_ref(X, y, mode="lbfgs", cov_fct="exponential", gp_approx="vecchia", num_neighbors=30, ordering="random",
                 cov_pars="0.1,1.0,0.1")
    la = run_ref(X, y, mode="eval", cov_fct="exponential", gp_approx="vecchia_latent", likelihood="gaussian",
                 matrix_inversion_method="iterative", num_neighbors=30, ordering="random", cov_pars="1.0,0.1",
                 aux_pars="0.1", cg_delta_conv="1e-2", num_rand_vec_trace="50", seed_rand_vec_trace="1")
    yb = synthetic.bench_bernoulli_y(X)
    lb = run_ref(X, yb, mode="eval", cov_fct="exponential", gp_approx="vecchia", likelihood="bernoulli_logit",
                 matrix_inversion_method="iterative", num_neighbors=30, ordering="random", cov_pars="1.0,0.1",
                 cg_delta_conv="1e-2", num_rand_vec_trace="50", seed_rand_vec_trace="1")
    out = {"bernoulli": dict(n=n, cov_pars=[1.0, 0.1], cg_delta_conv=1e-2, num_rand_vec_trace=50, nll=lb["nll"],
                             grad=lb["grad"]),
           "exact": dict(n=n, cov_pars=[0.1, 1.0, 0.1], nll=ex["nll"], grad=ex["grad"], sigma2=ex["sigma2"]),
           "latent": dict(n=n, cov_pars=[1.0, 0.1], aux=0.1, cg_delta_conv=1e-2, num_rand_vec_trace=50,
                          nll=la["nll"], grad=la["grad"])}
    print(out, file=sys.stderr)
    with open(os.path.join(HERE, "golden_100k.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
