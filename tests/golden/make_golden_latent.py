#!/usr/bin/env python3
"""Golden fixtures for the latent Vecchia + iterative-methods path, produced by the
REFERENCE (oracle/_ref/ref_harness built from /root/reference by oracle/Makefile).

    make -C oracle ref && python3 tests/golden/make_golden_latent.py

Each case evaluates the Laplace-approximated nll and its gradient
(CalcCovFactorOrModeAndNegLL + CalcGradPars) with matrix_inversion_method = "iterative"
and the VADU preconditioner, probes from seed_rand_vec_trace (first draw). Tight-tolerance
cases (cg_delta_conv = 1e-10) pin the arithmetic; default-tolerance cases (1e-2) pin the
stopping rules as well. Inputs are regenerated from the portable LCG generators.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from gpboost_amd import synthetic  # noqa: E402
from make_golden import run_ref  # noqa: E402


def main():
    cases = {}
    n = 2000
    X = synthetic.bench_coords(n)
    yg = synthetic.bench_gaussian_y(n)
    yb = synthetic.bench_bernoulli_y(X)
    rX, ry_probit = synthetic.rtest_bernoulli_probit_y(100)
    specs = [
        # name, data, likelihood, cov_fct, shape, m, cov_pars, aux, cg_delta_conv, t, seed
        ("gauss_m30_exp_tight", "bench", "gaussian", "exponential", 0.5, 30, [1.0, 0.1], 0.1, 1e-10, 50, 1),
        ("gauss_m30_exp_default", "bench", "gaussian", "exponential", 0.5, 30, [1.0, 0.1], 0.1, 1e-2, 50, 1),
        ("gauss_m20_matern15_t20", "bench", "gaussian", "matern", 1.5, 20, [0.8, 0.15], 0.3, 1e-6, 20, 3),
        ("bern_m30_exp_tight", "bench_bern", "bernoulli_logit", "exponential", 0.5, 30, [1.0, 0.1], None, 1e-10, 50, 1),
        ("bern_m30_exp_default", "bench_bern", "bernoulli_logit", "exponential", 0.5, 30, [1.0, 0.1], None, 1e-2, 50, 1),
        ("bern_m10_gaussian_t30", "bench_bern", "bernoulli_logit", "gaussian", 0.5, 10, [1.5, 0.2], None, 1e-4, 30, 5),
        ("bern_m16_matern25", "bench_bern", "bernoulli_logit", "matern", 2.5, 16, [0.6, 0.08], None, 1e-3, 50, 1),
        ("rtest_bern_m30_exp", "rtest_bern", "bernoulli_logit", "exponential", 0.5, 30, [1.0, 0.2], None, 1e-8, 50, 1),
    ]
    for name, data, lik, cov, shape, m, cp, aux, dc, t, seed in specs:
        if data == "bench":
            coords, y = X, yg
        elif data == "bench_bern":
            coords, y = X, yb
        else:
            coords, y = rX, ry_probit
        opts = dict(cov_fct=cov, shape=shape, num_neighbors=m, ordering="random", likelihood=lik,
                    matrix_inversion_method="iterative", cov_pars=",".join(repr(float(v)) for v in cp),
                    cg_delta_conv=repr(dc), num_rand_vec_trace=t, seed_rand_vec_trace=seed)
        if lik == "gaussian":
            opts["gp_approx"] = "vecchia_latent"
            opts["aux_pars"] = repr(float(aux))
        else:
            opts["gp_approx"] = "vecchia"
        r = run_ref(coords, y, **opts)
        cases[name] = dict(data=data, n=int(coords.shape[0]), likelihood=lik, cov_fct=cov, shape=shape,
                           num_neighbors=m, cov_pars=cp, aux=aux, cg_delta_conv=dc, num_rand_vec_trace=t,
                           seed_rand_vec_trace=seed, nll=r["nll"], grad=r["grad"])
        print(name, r["nll"], r["grad"], file=sys.stderr)
    with open(os.path.join(HERE, "golden_latent.json"), "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
