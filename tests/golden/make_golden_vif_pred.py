#!/usr/bin/env python3
"""Reference fixtures for predictions with the full-scale Vecchia approximation ("VIF", gp_approx =
"full_scale_vecchia", Gaussian likelihood): CalcPredVecchiaObservedFirstOrder's full-scale branches
(Vecchia_utils.cpp:1634-1980, re_model_template.h:3708-3792) from the reference itself (oracle/_ref/ref_harness):

    make -C oracle ref && python3 tests/golden/make_golden_vif_pred.py

Per case: predictive means with variances or the covariance matrix (latent process or response) for
vecchia_pred_type order_obs_first_cond_obs_only / order_obs_first_cond_all, at given parameters; prediction
points from the portable LCG (the first five on training coordinates for cond_obs_only).
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, fmt_pars, run_ref  # noqa: E402

sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from gpboost_amd import synthetic  # noqa: E402

OUT = os.path.join(HERE, "golden_vif_pred.json")


def pred_points(X, npred, dup):
    xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    if dup:
        xp[:5] = X[:5]
    return xp


def main():
    out = {}
    cases = [
        # name, n, m, nn, cov_fct, shape, cov_pars, npred, ptype, nn_pred, opts
        ("obs_only_var", 1500, 60, 10, "exponential", 0.5, [0.1, 1.0, 0.1], 40, "order_obs_first_cond_obs_only", -1,
         dict(predict_var="1")),
        ("obs_only_cov_resp", 1500, 60, 10, "exponential", 0.5, [0.1, 1.0, 0.1], 40, "order_obs_first_cond_obs_only",
         -1, dict(predict_cov="1", predict_response="1")),
        ("obs_only_var_m15_nn30", 2000, 100, 30, "matern", 1.5, [0.2, 0.8, 0.15], 50, "order_obs_first_cond_obs_only",
         -1, dict(predict_var="1", predict_response="1")),
        ("cond_all_cov", 1200, 50, 10, "exponential", 0.5, [0.1, 1.0, 0.1], 30, "order_obs_first_cond_all", -1,
         dict(predict_cov="1")),
        ("cond_all_var_nnp12", 1200, 50, 8, "gaussian", 0.5, [0.15, 1.2, 0.08], 30, "order_obs_first_cond_all", 12,
         dict(predict_var="1")),
    ]
    for name, n, m, nn, cov, shape, cp, npred, ptype, nnp, opts in cases:
        X = synthetic.bench_coords(n)
        y = synthetic.bench_spatial_gaussian_y(X)
        dup = ptype.endswith("obs_only")
        xp = pred_points(X, npred, dup)
        spec = dict(cov_fct=cov, shape=str(shape), gp_approx="full_scale_vecchia", num_ind_points=m, num_neighbors=nn,
                    ind_points_selection="kmeans++", seed=0, ordering="random")
        path = os.path.join(HERE, "_vif_pred_tmp.bin")
        with open(path, "wb") as f:
            f.write(np.array([npred], dtype=np.int32).tobytes())
            f.write(np.asfortranarray(xp).T.astype(np.float64).tobytes())
        try:
            r = run_ref(X, y, cov_pars=fmt_pars(cp), mode="predict", pred=path, vecchia_pred_type=ptype,
                        num_neighbors_pred=nnp, **opts, **spec)
        finally:
            os.unlink(path)
        c = dict(n=n, m=m, num_neighbors=nn, cov_pars=cp, npred=npred, dup5=dup, vecchia_pred_type=ptype,
                 num_neighbors_pred=nnp, response=opts.get("predict_response") == "1", spec=spec, mean=r["mean"])
        for k in ("var", "cov"):
            if k in r:
                c[k] = r[k]
        out[name] = c
        print(name, r["mean"][:3], file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
