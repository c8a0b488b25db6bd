#!/usr/bin/env python3
"""Reference fixtures for the Gaussian Vecchia prediction types order_obs_first_cond_all (prediction
points condition on the observed AND the earlier prediction points: CalcPredVecchiaObservedFirstOrder
with CondObsOnly = false, Vecchia_utils.cpp:1634-2006) and order_pred_first (prediction points first:
CalcPredVecchiaPredictedFirstOrder, :2018-2239), from the reference itself
(oracle/_ref/ref_harness mode=predict vecchia_pred_type=order_obs_first_cond_all): predictive means,
variances and the full covariance matrix, latent and response scale. Build container only:

    make -C oracle ref && python3 tests/golden/make_golden_pred_types.py
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

OUT = os.path.join(HERE, "golden_pred_types.json")


def pred_coords(npred, d=2):
    return synthetic.lcg_unif(npred * d, 0.713).reshape(d, npred).T.copy()


def case(n, npred, cov_pars, m=30, mp=None, cov=False, response=False, cov_fct="exponential", shape=0.5,
         ptype="order_obs_first_cond_all", gp_approx="vecchia"):
    X = synthetic.bench_coords(n)
    y = synthetic.bench_spatial_gaussian_y(X)
    Xp = pred_coords(npred)
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([npred], dtype=np.int32).tobytes())
        f.write(np.asfortranarray(Xp).T.astype(np.float64).tobytes())
        ppath = f.name
    spec = dict(cov_fct=cov_fct, shape=str(shape), gp_approx=gp_approx, num_neighbors=m, ordering="random")
    extra = dict(vecchia_pred_type=ptype) if gp_approx == "vecchia" else {}
    if mp:
        extra["num_neighbors_pred"] = str(mp)
    if cov:
        extra["predict_cov"] = "1"
    else:
        extra["predict_var"] = "1"
    if response:
        extra["predict_response"] = "1"
    try:
        r = run_ref(X, y, cov_pars=fmt_pars(cov_pars), mode="predict", pred=ppath, **spec, **extra)
    finally:
        os.unlink(ppath)
    out = dict(n=n, npred=npred, cov_pars=list(cov_pars), spec=spec, mp=mp, response=response, ptype=ptype,
               mean=r["mean"])
    out["cov" if cov else "var"] = r["cov" if cov else "var"]
    return out


def main():
    cases = {
        "cond_all_var": case(2000, 400, (0.1, 1.0, 0.1)),
        "cond_all_var_resp": case(2000, 400, (0.1, 1.0, 0.1), response=True),
        "cond_all_cov": case(1500, 150, (0.2, 0.8, 0.15), m=20, mp=25, cov=True),
        "cond_all_matern_var": case(2000, 300, (0.05, 1.2, 0.2), m=25, cov_fct="matern", shape=1.5),
        # order_pred_first (CalcPredVecchiaPredictedFirstOrder, Vecchia_utils.cpp:2018-2239)
        "pred_first_var": case(2000, 300, (0.1, 1.0, 0.1), ptype="order_pred_first"),
        "pred_first_var_resp": case(2000, 300, (0.1, 1.0, 0.1), response=True, ptype="order_pred_first"),
        "pred_first_cov": case(1500, 150, (0.2, 0.8, 0.15), m=20, mp=25, cov=True, ptype="order_pred_first"),
        "pred_first_matern_var": case(2000, 300, (0.05, 1.2, 0.2), m=25, cov_fct="matern", shape=1.5,
                                      ptype="order_pred_first"),
        # latent_order_obs_first_cond_* with the Gaussian likelihood (CalcPredVecchiaLatentObservedFirstOrder,
        # Vecchia_utils.cpp:2241-2442)
        "latent_gauss_obs_only_var": case(1500, 200, (0.1, 1.0, 0.1), m=20,
                                          ptype="latent_order_obs_first_cond_obs_only"),
        "latent_gauss_cond_all_var": case(1500, 200, (0.1, 1.0, 0.1), m=20, ptype="latent_order_obs_first_cond_all"),
        "latent_gauss_cond_all_resp": case(1500, 200, (0.1, 1.0, 0.1), m=20, response=True,
                                           ptype="latent_order_obs_first_cond_all"),
        "latent_gauss_cond_all_cov": case(1000, 100, (0.2, 0.8, 0.15), m=15, mp=20, cov=True,
                                          ptype="latent_order_obs_first_cond_all"),
        "latent_gauss_matern_cond_all_var": case(1500, 200, (0.05, 1.2, 0.2), m=20, cov_fct="matern", shape=1.5,
                                                 ptype="latent_order_obs_first_cond_all"),
        # gp_approx = "none" (CalcPred, the exact conditional Gaussian)
        "dense_var": case(1500, 200, (0.1, 1.0, 0.1), gp_approx="none", ptype=None),
        "dense_var_resp": case(1500, 200, (0.1, 1.0, 0.1), gp_approx="none", response=True, ptype=None),
        "dense_cov_matern": case(1000, 100, (0.05, 1.2, 0.2), cov_fct="matern", shape=1.5, cov=True, gp_approx="none",
                                 ptype=None),
    }
    for k, v in cases.items():
        print(k, v["mean"][:3], file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f)


if __name__ == "__main__":
    main()
