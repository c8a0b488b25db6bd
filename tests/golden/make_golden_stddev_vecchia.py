#!/usr/bin/env python3
"""Reference fixtures for the standard deviations of the covariance parameters of the Gaussian Vecchia
model (GPB_GetCovPar(calc_std_dev = true) -> CalcStdDevCovPar, re_model_template.h:9775-9789 ->
CalcFisherInformation_Vecchia :9238-9307, the default stochastic-trace form with probes from
GenRandVecNormalParallel(seed_rand_vec_trace, cg_generator_counter_ = 0)) from the reference itself
(oracle/_ref/ref_harness, mode=stddev):

    make -C oracle ref && python3 tests/golden/make_golden_stddev_vecchia.py

Inputs are regenerated from the portable LCG generators (gpboost_amd/synthetic.py). Cases cover the four
covariance functions, both orderings, several probe counts / seeds, and n = 20000 (beyond the dense and
LDS-segment heads of the GPU solve plan, so its level-scheduled tail runs).
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, fmt_pars, run_ref  # noqa: E402

sys.path.insert(0, ROOT)
from gpboost_amd import synthetic  # noqa: E402

OUT = os.path.join(HERE, "golden_stddev_vecchia.json")


def case(n, nn, cov_pars, cov_fct="exponential", shape=0.5, ordering="random", seed=0, t=None, seed_rv=None):
    X = synthetic.bench_coords(n)
    y = synthetic.bench_spatial_gaussian_y(X)
    spec = dict(cov_fct=cov_fct, shape=str(shape), gp_approx="vecchia", num_neighbors=nn, ordering=ordering,
                seed=seed)
    opts = dict(spec)
    if t is not None or seed_rv is not None:
        opts["num_rand_vec_trace"] = 50 if t is None else t
        opts["seed_rand_vec_trace"] = 1 if seed_rv is None else seed_rv
    r = run_ref(X, y, mode="stddev", cov_pars=fmt_pars(cov_pars), **opts)
    return dict(n=n, num_neighbors=nn, spec=spec, num_rand_vec_trace=t, seed_rand_vec_trace=seed_rv,
                cov_pars=r["cov_pars"], std_dev=r["std_dev"])


def main():
    cases = {
        "sdv_exp_n2000_nn20": case(2000, 20, (0.25, 1.0, 0.1)),
        "sdv_exp_n2000_nn20_t10": case(2000, 20, (0.25, 1.0, 0.1), t=10),
        "sdv_matern15_n3000_nn30": case(3000, 30, (0.2, 1.3, 0.15), cov_fct="matern", shape=1.5),
        "sdv_matern25_n2000_nn10_seed7": case(2000, 10, (0.1, 0.9, 0.05), cov_fct="matern", shape=2.5, seed_rv=7),
        "sdv_gauss_n1500_nn15_t20": case(1500, 15, (0.3, 0.8, 0.2), cov_fct="gaussian", shape=0.0, t=20),
        "sdv_exp_n1000_nn8_none": case(1000, 8, (0.25, 0.7, 0.05), ordering="none"),
        "sdv_exp_n20000_nn30": case(20000, 30, (0.25, 1.0, 0.1), seed=3),
    }
    for k, v in cases.items():
        print(k, v["std_dev"], file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
