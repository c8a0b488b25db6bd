#!/usr/bin/env python3
"""Laplace predictive variances / covariances pinned to the reference's own draws: the reference run on ONE
thread (oracle/_ref/ref_harness threads=1), where PredictLaplaceApproxVecchia (likelihoods.h:6668-6700) draws
from a single mt19937 seeded by unif{0..2147483646}(cg_generator_) of the likelihood's default-seeded
generator, z1_j / z2_j interleaved per draw. gpboost_amd reproduces that stream with
GPBOOST_AMD_PRED_DRAWS=reference, so the simulated moments agree to the CG tolerance (cg_delta_conv = 1e-10
here) instead of to the statistical 6-standard-error bound.

    make -C oracle ref && python3 tests/golden/make_golden_latent_pred_1t.py
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from gpboost_amd import synthetic  # noqa: E402
from make_golden import fmt_pars, run_ref  # noqa: E402

OUT = os.path.join(HERE, "golden_latent_pred_1t.json")


def data(lik, n):
    X = synthetic.bench_coords(n)
    return X, (synthetic.bench_poisson_y(X) if lik == "poisson" else synthetic.bench_bernoulli_y(X))


def case(lik, n, npred, cov_pars, nsim, ptype, cov=False, response=False, m=20):
    X, y = data(lik, n)
    Xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([npred], dtype=np.int32).tobytes())
        f.write(np.asfortranarray(Xp).T.astype(np.float64).tobytes())
        ppath = f.name
    spec = dict(cov_fct="exponential", gp_approx="vecchia", likelihood=lik, num_neighbors=m, ordering="random",
                matrix_inversion_method="iterative", num_rand_vec_trace=20, cg_delta_conv="1e-10", threads=1,
                vecchia_pred_type=ptype, nsim_var_pred=str(nsim))
    extra = {"predict_cov": "1"} if cov else {"predict_var": "1"}
    if response:
        extra["predict_response"] = "1"
    try:
        r = run_ref(X, y, cov_pars=fmt_pars(cov_pars), mode="predict", pred=ppath, **spec, **extra)
    finally:
        os.unlink(ppath)
    out = dict(lik=lik, n=n, npred=npred, cov_pars=list(cov_pars), nsim=nsim, ptype=ptype, response=response, m=m,
               mean=r["mean"])
    out["cov" if cov else "var"] = r["cov" if cov else "var"]
    return out


def main():
    cases = {
        "bern_obs_only_var": case("bernoulli_logit", 2000, 60, (1.0, 0.1), 100, "latent_order_obs_first_cond_obs_only"),
        "bern_cond_all_cov": case("bernoulli_logit", 1500, 40, (1.2, 0.15), 64, "latent_order_obs_first_cond_all",
                                  cov=True),
        "pois_obs_only_resp": case("poisson", 2000, 50, (0.8, 0.1), 80, "latent_order_obs_first_cond_obs_only",
                                   response=True),
        "probit_cond_all_var": case("bernoulli_probit", 1200, 30, (1.0, 0.2), 50, "latent_order_obs_first_cond_all"),
    }
    for k, v in cases.items():
        print(k, v["mean"][:2], (v.get("var") or v.get("cov"))[:2], file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f)


if __name__ == "__main__":
    main()
