#!/usr/bin/env python3
"""Reference fixtures for combined Gaussian process + grouped random effects models (gp_approx = "none",
Gaussian likelihood; re_model_template.h:236-239 allows grouped effects beside a GP only without an
approximation) from the reference itself (oracle/_ref/ref_harness with group labels):

    make -C oracle ref && python3 tests/golden/make_golden_combined.py

Per case: nll and gradient with the nugget as a parameter ("eval") and profiled out ("lbfgs"), default fits
(GPB_OptimCovPar, lbfgs), and predictions (means, variances / covariance matrices) at new coordinates with
seen and new labels. Inputs: gpboost_amd.synthetic (bench_coords, bench_groups, and the R tests' combined data).
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

OUT = os.path.join(HERE, "golden_combined.json")


def data(kind, n, levels):
    if kind == "rtest":
        X, g, y = synthetic.rtest_combined_y(n)
        return X, g.reshape(-1, 1), y
    X = synthetic.bench_coords(n)
    g = synthetic.bench_groups(n, levels)
    y = synthetic.bench_spatial_gaussian_y(X) + synthetic.bench_grouped_y(g, noise_sd=0.3)
    return X, g, y


def spec(cov_fct, shape):
    return dict(cov_fct=cov_fct, shape=str(shape), gp_approx="none")


def case(kind, n, levels, cov_pars, cov_fct="exponential", shape=0.5):
    X, g, y = data(kind, n, levels)
    sp = spec(cov_fct, shape)
    ev = run_ref(X, y, groups=g, cov_pars=fmt_pars(cov_pars), mode="eval", **sp)
    lb = run_ref(X, y, groups=g, cov_pars=fmt_pars(cov_pars), mode="lbfgs", **sp)
    return dict(kind=kind, n=n, levels=list(levels), cov_pars=list(cov_pars), spec=sp, nll=ev["nll"], grad=ev["grad"],
                lbfgs_nll=lb["nll"], lbfgs_grad=lb["grad"], lbfgs_sigma2=lb["sigma2"])


def fit_case(kind, n, levels, cov_fct="exponential", shape=0.5):
    X, g, y = data(kind, n, levels)
    sp = spec(cov_fct, shape)
    r = run_ref(X, y, groups=g, mode="fit", **sp)
    return dict(kind=kind, n=n, levels=list(levels), spec=sp, **{k: r[k] for k in r if k not in ("ok", "n", "d")})


def pred_case(kind, n, levels, cov_pars, npred, cov=False, response=False, cov_fct="exponential", shape=0.5):
    X, g, y = data(kind, n, levels)
    K = g.shape[1]
    Xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    gp = np.array([[g[(7 * j) % n, k] if j % 3 else 100000 + j // 2 for k in range(K)] for j in range(npred)],
                  dtype=np.int64)
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([npred], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(Xp.T).astype(np.float64).tobytes())
        f.write(np.ascontiguousarray(gp.T).astype(np.int32).tobytes())
        ppath = f.name
    extra = {"predict_cov" if cov else "predict_var": "1"}
    if response:
        extra["predict_response"] = "1"
    sp = spec(cov_fct, shape)
    try:
        r = run_ref(X, y, groups=g, cov_pars=fmt_pars(cov_pars), mode="predict", pred=ppath, **sp, **extra)
    finally:
        os.unlink(ppath)
    out = dict(kind=kind, n=n, levels=list(levels), cov_pars=list(cov_pars), spec=sp, npred=npred, response=response,
               coords_pred=Xp.tolist(), labels=gp.tolist(), mean=r["mean"])
    out["cov" if cov else "var"] = r["cov" if cov else "var"]
    return out


def main():
    cases = {
        "cb_rtest_k1": case("rtest", 100, (10,), (0.05, 0.6, 1.0, 0.1)),
        "cb_k1_n500_exp": case("bench", 500, (40,), (0.1, 0.5, 1.0, 0.1)),
        "cb_k2_n2000_matern15": case("bench", 2000, (100, 12), (0.1, 0.8, 0.3, 1.2, 0.15), "matern", 1.5),
        "cb_k1_n1500_gauss": case("bench", 1500, (60,), (0.2, 0.4, 0.9, 0.2), "gaussian", 0.0),
        "fit_cb_rtest_k1": fit_case("rtest", 100, (10,)),
        "fit_cb_k1_n500_exp": fit_case("bench", 500, (40,)),
        "fit_cb_k2_n1200_matern25": fit_case("bench", 1200, (50, 7), "matern", 2.5),
        "pred_cb_k1_var_resp": pred_case("bench", 500, (40,), (0.1, 0.5, 1.0, 0.1), 30, response=True),
        "pred_cb_k2_cov": pred_case("bench", 2000, (100, 12), (0.1, 0.8, 0.3, 1.2, 0.15), 24, cov=True,
                                    cov_fct="matern", shape=1.5),
        "pred_cb_rtest_cov": pred_case("rtest", 100, (10,), (0.0226, 0.6147, 1.0245, 0.1118), 12, cov=True),
    }
    for k, v in cases.items():
        print(k, v.get("nll"), v.get("grad", v.get("cov_pars")), v.get("num_it"), file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f)


if __name__ == "__main__":
    main()
