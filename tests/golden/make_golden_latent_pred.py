#!/usr/bin/env python3
"""Golden fixtures for latent-model Vecchia predictions from the reference itself
(oracle/_ref/ref_harness mode=predict: GPB_SetPredictionData + Predict, re_model.cpp:927 ->
re_model_template.h:3146 -> CalcPredVecchiaObservedFirstOrder Vecchia_utils.cpp:1634 +
PredictLaplaceApproxVecchia likelihoods.h:6576). The default prediction type of latent models is
latent_order_obs_first_cond_obs_only; the mode is found from zero at the given parameters
(re_model.cpp:967-977). Means are deterministic given the mode; the iterative predictive variances
are a simulation (nsim_var_pred draws from the reference's thread-seeded generators), so the
fixtures hold them at a large nsim as the statistical target.

    make -C oracle ref && python3 tests/golden/make_golden_latent_pred.py [--big]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from gpboost_amd import synthetic  # noqa: E402
from make_golden import fmt_pars, run_ref  # noqa: E402

OUT = os.path.join(HERE, "golden_latent_pred.json")


def pred_coords(npred, d=2):
    return synthetic.lcg_unif(npred * d, 0.713).reshape(d, npred).T.copy()


def case(n, npred, lik, cov_pars, nu=0, m=20, t=50, nsim=None, response=False, cov=False, **opts):
    X = synthetic.repeated_coords(n, nu) if nu else synthetic.bench_coords(n)
    y = synthetic.bench_bernoulli_y(X) if lik == "bernoulli_logit" else synthetic.bench_gaussian_y(n)
    Xp = pred_coords(npred)
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([npred], dtype=np.int32).tobytes())
        f.write(np.asfortranarray(Xp).T.astype(np.float64).tobytes())
        ppath = f.name
    spec = dict(cov_fct="exponential", gp_approx="vecchia" if lik == "bernoulli_logit" else "vecchia_latent",
                likelihood=lik, num_neighbors=m, ordering="random", matrix_inversion_method="iterative",
                num_rand_vec_trace=t)
    spec.update(opts)
    try:
        extra = dict(predict_var="1", nsim_var_pred=str(nsim)) if nsim else {}
        if cov:
            extra = dict(predict_cov="1", nsim_var_pred=str(nsim))
        if response:
            extra["predict_response"] = "1"
        r = run_ref(X, y, cov_pars=fmt_pars(cov_pars), mode="predict", pred=ppath, **spec, **extra)
    finally:
        os.unlink(ppath)
    out = dict(n=n, nu=nu, npred=npred, lik=lik, cov_pars=list(cov_pars), spec=spec, mean=r["mean"], response=response)
    if nsim:
        out.update(nsim=nsim)
        out["cov" if cov else "var"] = r["cov" if cov else "var"]
    return out


def main():
    cases = json.load(open(OUT)) if os.path.exists(OUT) else {}
    tight = dict(cg_delta_conv="1e-10")
    if "--new" in sys.argv:
        # predictive covariance (obs-only) and latent_order_obs_first_cond_all (PredictLaplaceApproxVecchia
        # with CondObsOnly = false, likelihoods.h:6610-6749)
        cases["bern_n2000_tight_cov"] = case(2000, 40, "bernoulli_logit", (1.0, 0.1), nsim=20000, cov=True, **tight)
        cases["bern_n2000_tight_condall"] = case(2000, 300, "bernoulli_logit", (1.0, 0.1), nsim=20000,
                                                 vecchia_pred_type="latent_order_obs_first_cond_all", **tight)
        cases["gauss_n2000_tight_condall"] = case(2000, 300, "gaussian", (1.0, 0.1), aux_pars="0.1", nsim=20000,
                                                  vecchia_pred_type="latent_order_obs_first_cond_all", **tight)
        cases["bern_n2000_tight_condall_cov"] = case(2000, 40, "bernoulli_logit", (1.0, 0.1), nsim=20000, cov=True,
                                                     vecchia_pred_type="latent_order_obs_first_cond_all", **tight)
    elif "--big" not in sys.argv:
        cases["bern_n2000_tight"] = case(2000, 300, "bernoulli_logit", (1.0, 0.1), nsim=20000, **tight)
        cases["bern_n2000_default"] = case(2000, 300, "bernoulli_logit", (1.0, 0.1))
        cases["gauss_n2000_tight"] = case(2000, 300, "gaussian", (1.0, 0.1), aux_pars="0.1", nsim=20000, **tight)
        cases["bern_rep_n3000_tight"] = case(3000, 200, "bernoulli_logit", (0.8, 0.2), nu=1200, m=15, **tight)
        # response probabilities (adaptive Gauss-Hermite over the simulated latent variances)
        cases["bern_n2000_tight_response"] = case(2000, 300, "bernoulli_logit", (1.0, 0.1), nsim=20000,
                                                  response=True, **tight)
    else:
        cases["bern_n100k_default"] = case(100000, 5000, "bernoulli_logit", (1.0, 0.1), m=30)
    for k, v in cases.items():
        print(k, v["mean"][:3], v.get("var", v.get("cov", [None]))[:3], file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
