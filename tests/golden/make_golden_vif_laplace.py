#!/usr/bin/env python3
"""Reference fixtures for the full-scale Vecchia approximation ("VIF", gp_approx = "full_scale_vecchia") with a
non-Gaussian likelihood and matrix_inversion_method = "cholesky" (the reference's FSVA Laplace approximation:
FindModePostRandEffCalcMLLFSVA likelihoods.h:2316-2742, CalcGradNegMargLikelihoodLaplaceApproxFSVA :3886-4925,
PredictLaplaceApproxFSVA :6060-6551), from the reference itself (oracle/_ref/ref_harness built from
/root/reference by oracle/Makefile):

    make -C oracle ref && python3 tests/golden/make_golden_vif_laplace.py

Cases: nll + gradient for bernoulli_logit / bernoulli_probit / poisson / gamma (shape gradient) over four
covariance functions (kmeans++ inducing points: the reference refuses 'random' for non-Gaussian data), m = 20-200 inducing points and 8-30 neighbours at n = 1000-3000 (with the reference's
ordering, inducing points and neighbour lists for the small cases), one bernoulli_logit evaluation at n = 20000,
L-BFGS fits, the gradient wrt fixed effects and latent predictions (means, variances, covariance matrices).
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
import numpy as np  # noqa: E402

from gpboost_amd import synthetic  # noqa: E402

OUT = os.path.join(HERE, "golden_vif_laplace.json")


def data(kind, n):
    X = synthetic.bench_coords(n)
    if kind == "bench_gamma":
        return X, synthetic.bench_gamma_y(X)
    if kind == "bench_pois":
        return X, synthetic.bench_poisson_y(X)
    return X, synthetic.bench_bernoulli_y(X)


def spec(lik, cov_fct, shape, m, nn, sel="kmeans++", seed=0, aux=None):
    s = dict(cov_fct=cov_fct, shape=str(shape), gp_approx="full_scale_vecchia", num_ind_points=m, num_neighbors=nn,
             ind_points_selection=sel, seed=seed, ordering="random", likelihood=lik,
             matrix_inversion_method="cholesky")
    if aux is not None:
        s["aux_pars"] = repr(float(aux))
    return s


def main():
    out = {}
    evals = [
        # name, data, n, likelihood, cov_fct, shape, m, nn, cov_pars, aux, sel, seed, dump
        ("logit_exp_m50_nn10", "bench_bern", 2000, "bernoulli_logit", "exponential", 0.5, 50, 10, [1.0, 0.1], None,
         "kmeans++", 0, True),
        ("probit_exp_m50_nn10", "bench_bern", 2000, "bernoulli_probit", "exponential", 0.5, 50, 10, [1.0, 0.1], None,
         "kmeans++", 0, True),
        ("pois_matern15_m100_nn20", "bench_pois", 2000, "poisson", "matern", 1.5, 100, 20, [0.8, 0.15], None,
         "kmeans++", 0, True),
        ("gamma_exp_m40_nn15", "bench_gamma", 2000, "gamma", "exponential", 0.5, 40, 15, [1.0, 0.1], 2.0,
         "kmeans++", 0, True),
        ("logit_gaussian_m60_nn15_seed3", "bench_bern", 1500, "bernoulli_logit", "gaussian", 0.5, 60, 15, [1.5, 0.04],
         None, "kmeans++", 3, True),
        ("logit_matern25_m200_nn30", "bench_bern", 3000, "bernoulli_logit", "matern", 2.5, 200, 30, [0.6, 0.08], None,
         "kmeans++", 7, True),
        ("pois_exp_m20_nn8", "bench_pois", 1000, "poisson", "exponential", 0.5, 20, 8, [0.9, 0.12], None,
         "kmeans++", 0, True),
        ("logit_exp_m200_nn30_n20000", "bench_bern", 20000, "bernoulli_logit", "exponential", 0.5, 200, 30, [1.0, 0.1],
         None, "kmeans++", 0, False),
    ]
    for name, kind, n, lik, cov, shape, m, nn, cp, aux, sel, seed, dump in evals:
        X, y = data(kind, n)
        sp = spec(lik, cov, shape, m, nn, sel, seed, aux)
        r = run_ref(X, y, cov_pars=fmt_pars(cp), mode="eval", dump_nn=int(dump), **sp)
        c = dict(kind="eval", data=kind, n=n, spec=sp, cov_pars=cp, aux=aux, nll=r["nll"], grad=r["grad"],
                 ind_points=r["ind_points"], ref_seconds=r["median_time"])
        if dump:
            c["perm"] = r["perm"]
            c["neighbors"] = r["neighbors"]
            c["D_inv"] = r["D_inv"]
        out[name] = c
        print(name, r["nll"], r["grad"], r["median_time"], file=sys.stderr)
    # L-BFGS fits (FindInitCovPar start, the Python package's default optimizer settings)
    for fname, kind, n, lik, m, nn in [("fit_logit_m30_nn10_n800", "bench_bern", 800, "bernoulli_logit", 30, 10),
                                        ("fit_pois_m20_nn8_n600", "bench_pois", 600, "poisson", 20, 8)]:
        X, y = data(kind, n)
        sp = spec(lik, "exponential", 0.5, m, nn)
        r = run_ref(X, y, mode="fit", **sp)
        out[fname] = dict(kind="fit", data=kind, n=n, spec=sp, init_cov_pars=r["init_cov_pars"], cov_pars=r["cov_pars"],
                          nll=r["nll"], num_it=r["num_it"])
        print(fname, r["cov_pars"], r["num_it"], file=sys.stderr)
    # gradient wrt the fixed effects F at the mode (CalcGradientF)
    X, y = data("bench_pois", 1000)
    fe = 0.3 * np.sin(3.0 * X[:, 0]) - 0.2
    sp = spec("poisson", "exponential", 0.5, 30, 10)
    cp = [0.9, 0.12]
    r = run_ref(X, y, fe=fe, cov_pars=fmt_pars(cp), mode="eval", **sp)
    rg = run_ref(X, y, fe=fe, cov_pars=fmt_pars(cp), mode="grad_f", **sp)
    out["gradf_pois_m30_nn10_n1000"] = dict(kind="gradf", data="bench_pois", n=1000, spec=sp, cov_pars=cp,
                                            nll=r["nll"], grad=r["grad"], grad_f=rg["grad_f"])
    # latent predictions: means / variances (cond_obs_only), covariance (cond_all), response probabilities
    X, y = data("bench_bern", 1000)
    npred = 40
    cp = [1.0, 0.1]
    for pname, ptype, opts in [("pred_var_obs_only", "latent_order_obs_first_cond_obs_only", dict(predict_var="1")),
                               ("pred_cov_obs_only", "latent_order_obs_first_cond_obs_only", dict(predict_cov="1")),
                               ("pred_cov_cond_all", "latent_order_obs_first_cond_all", dict(predict_cov="1")),
                               ("pred_var_cond_all", "latent_order_obs_first_cond_all", dict(predict_var="1")),
                               ("pred_resp_obs_only", "latent_order_obs_first_cond_obs_only",
                                dict(predict_var="1", predict_response="1"))]:
        sp = spec("bernoulli_logit", "exponential", 0.5, 30, 10)
        xq = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
        with open(os.path.join(HERE, "_pred_tmp.bin"), "wb") as f:
            f.write(np.array([npred], dtype=np.int32).tobytes())
            f.write(np.asfortranarray(xq).T.astype(np.float64).tobytes())
        try:
            r = run_ref(X, y, cov_pars=fmt_pars(cp), mode="predict", pred=os.path.join(HERE, "_pred_tmp.bin"),
                        vecchia_pred_type=ptype, **opts, **sp)
        finally:
            os.unlink(os.path.join(HERE, "_pred_tmp.bin"))
        c = dict(kind="pred", data="bench_bern", n=1000, npred=npred, spec=sp, cov_pars=cp, vecchia_pred_type=ptype,
                 response=opts.get("predict_response") == "1", mean=r["mean"])
        if "var" in r:
            c["var"] = r["var"]
        if "cov" in r:
            c["cov"] = r["cov"]
        out[pname] = c
        print(pname, r["mean"][:3], file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
