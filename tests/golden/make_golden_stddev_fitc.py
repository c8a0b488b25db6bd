#!/usr/bin/env python3
"""Reference fixtures for the standard deviations of the covariance parameters of the Gaussian FITC model
(GPB_GetCovPar(calc_std_dev = true) -> CalcStdDevCovPar, re_model_template.h:9775-9789 ->
CalcFisherInformation_FITC_FSA :9363-9548, gp_approx = "fitc", cholesky: Hutchinson estimates with probes
from GenRandVecNormalParallel(seed_rand_vec_trace, cg_generator_counter_ = 0)) from the reference itself
(oracle/_ref/ref_harness, mode=stddev):

    make -C oracle ref && python3 tests/golden/make_golden_stddev_fitc.py

Inputs are regenerated from the portable LCG generators (gpboost_amd/synthetic.py).
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

OUT = os.path.join(HERE, "golden_stddev_fitc.json")


def case(n, m, cov_pars, cov_fct="exponential", shape=0.5, sel="kmeans++", seed=0, t=None, seed_rv=None):
    X = synthetic.bench_coords(n)
    y = synthetic.bench_spatial_gaussian_y(X)
    spec = dict(cov_fct=cov_fct, shape=str(shape), gp_approx="fitc", num_ind_points=m, ind_points_selection=sel,
                seed=seed)
    opts = dict(spec)
    if t is not None or seed_rv is not None:
        opts["num_rand_vec_trace"] = 50 if t is None else t
        opts["seed_rand_vec_trace"] = 1 if seed_rv is None else seed_rv
    r = run_ref(X, y, mode="stddev", cov_pars=fmt_pars(cov_pars), **opts)
    return dict(n=n, m=m, spec=spec, num_rand_vec_trace=t, seed_rand_vec_trace=seed_rv, cov_pars=r["cov_pars"],
                std_dev=r["std_dev"])


def main():
    cases = {
        "sdf_exp_n2000_m50": case(2000, 50, (0.25, 1.0, 0.1)),
        "sdf_exp_n2000_m50_t10": case(2000, 50, (0.25, 1.0, 0.1), t=10),
        "sdf_matern15_n3000_m100": case(3000, 100, (0.2, 1.3, 0.15), cov_fct="matern", shape=1.5),
        "sdf_matern25_n1500_m60_seed7": case(1500, 60, (0.1, 0.9, 0.05), cov_fct="matern", shape=2.5, seed_rv=7),
        "sdf_gauss_n1500_m40_random_t20": case(1500, 40, (0.3, 0.8, 0.2), cov_fct="gaussian", shape=0.0, sel="random",
                                               seed=3, t=20),
        "sdf_exp_n20000_m200": case(20000, 200, (0.25, 1.0, 0.1)),
    }
    for k, v in cases.items():
        print(k, v["std_dev"], file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
