#!/usr/bin/env python3
"""Reference fixtures for the latent Vecchia path with matrix_inversion_method = "cholesky" (the reference's
exact Laplace-Vecchia branch: FindModePostRandEffCalcMLLVecchia / CalcGradNegMargLikelihoodLaplaceApproxVecchia /
PredictLaplaceApproxVecchia with the sparse Cholesky of Sigma^-1 + W, likelihoods.h:2935-2955, 3052-3070,
5207-5336, 6751-6811), from the reference itself (oracle/_ref/ref_harness built from /root/reference by
oracle/Makefile):

    make -C oracle ref && python3 tests/golden/make_golden_latent_chol.py

Cases: nll + gradient for bernoulli_logit / bernoulli_probit / poisson / gamma (shape gradient) and the
Gaussian "vecchia_latent" model (error-variance gradient) over four covariance functions and m = 10-30 at
n = 2000, one bernoulli_logit evaluation at n = 20000, the R tests' own data with num_neighbors = n - 1
(exact: test_GPModel_non_Gaussian_data.R:1196 probit 67.18342059, test_GPModel_gaussian_process.R:710-721
vecchia_latent cholesky 124.2549533), an L-BFGS fit, the gradient wrt fixed effects and latent / response
predictions. Inputs are regenerated from the portable LCG generators (gpboost_amd/synthetic.py).
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

OUT = os.path.join(HERE, "golden_latent_chol.json")


def data(kind, n):
    if kind == "rtest_probit":
        return synthetic.rtest_bernoulli_probit_y(n)
    if kind == "rtest_gauss":
        return synthetic.rtest_gaussian_y(n)
    X = synthetic.bench_coords(n)
    if kind == "bench_gamma":
        return X, synthetic.bench_gamma_y(X)
    if kind == "bench_pois":
        return X, synthetic.bench_poisson_y(X)
    if kind == "bench_gauss":
        return X, synthetic.bench_gaussian_y(n)
    return X, synthetic.bench_bernoulli_y(X)


def spec(lik, cov_fct, shape, m, ordering="random", aux=None):
    s = dict(cov_fct=cov_fct, shape=str(shape), num_neighbors=m, ordering=ordering, likelihood=lik,
             matrix_inversion_method="cholesky", gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia")
    if aux is not None:
        s["aux_pars"] = repr(float(aux))
    return s


def main():
    out = {}
    evals = [
        # name, data, n, likelihood, cov_fct, shape, m, cov_pars, aux, ordering, r_expected_nll
        ("logit_exp_m30", "bench_bern", 2000, "bernoulli_logit", "exponential", 0.5, 30, [1.0, 0.1], None, "random", None),
        ("probit_exp_m30", "bench_bern", 2000, "bernoulli_probit", "exponential", 0.5, 30, [1.0, 0.1], None, "random", None),
        ("pois_matern15_m20", "bench_pois", 2000, "poisson", "matern", 1.5, 20, [0.8, 0.15], None, "random", None),
        ("gamma_exp_m30", "bench_gamma", 2000, "gamma", "exponential", 0.5, 30, [1.0, 0.1], 2.0, "random", None),
        ("logit_gaussian_m10", "bench_bern", 2000, "bernoulli_logit", "gaussian", 0.5, 10, [1.5, 0.04], None, "random", None),
        ("logit_matern25_m16", "bench_bern", 2000, "bernoulli_logit", "matern", 2.5, 16, [0.6, 0.08], None, "random", None),
        ("gauss_latent_exp_m30", "bench_gauss", 2000, "gaussian", "exponential", 0.5, 30, [1.0, 0.1], 0.1, "random", None),
        ("gauss_latent_matern15_m20", "bench_gauss", 2000, "gaussian", "matern", 1.5, 20, [0.8, 0.15], 0.3, "random", None),
        ("rtest_probit_all", "rtest_probit", 100, "bernoulli_probit", "exponential", 0.5, 99, [1.0, 0.2], None, "none",
         67.18342059),
        ("rtest_gauss_latent_all", "rtest_gauss", 100, "gaussian", "exponential", 0.5, 99, [1.6, 0.2], 0.1, "none",
         124.2549533),
        ("logit_exp_m30_n20000", "bench_bern", 20000, "bernoulli_logit", "exponential", 0.5, 30, [1.0, 0.1], None, "random",
         None),
    ]
    for name, kind, n, lik, cov, shape, m, cp, aux, ordering, rexp in evals:
        X, y = data(kind, n)
        sp = spec(lik, cov, shape, m, ordering, aux)
        r = run_ref(X, y, cov_pars=fmt_pars(cp), mode="eval", **sp)
        out[name] = dict(kind="eval", data=kind, n=n, spec=sp, cov_pars=cp, aux=aux, nll=r["nll"], grad=r["grad"],
                         ref_seconds=r["median_time"])
        if rexp is not None:
            out[name]["r_expected_nll"] = rexp
        print(name, r["nll"], r["grad"], r["median_time"], file=sys.stderr)
    # L-BFGS fit (FindInitCovPar start, the Python package's default optimizer settings)
    X, y = data("bench_bern", 500)
    sp = spec("bernoulli_logit", "exponential", 0.5, 20)
    r = run_ref(X, y, mode="fit", **sp)
    out["fit_logit_m20_n500"] = dict(kind="fit", data="bench_bern", n=500, spec=sp, init_cov_pars=r["init_cov_pars"],
                                     cov_pars=r["cov_pars"], nll=r["nll"], num_it=r["num_it"])
    print("fit", r["cov_pars"], r["num_it"], file=sys.stderr)
    # gradient wrt the fixed effects F at the mode (CalcGradientF)
    X, y = data("bench_pois", 1000)
    fe = 0.3 * np.sin(3.0 * X[:, 0]) - 0.2
    sp = spec("poisson", "exponential", 0.5, 20)
    cp = [0.9, 0.12]
    r = run_ref(X, y, fe=fe, cov_pars=fmt_pars(cp), mode="eval", **sp)
    rg = run_ref(X, y, fe=fe, cov_pars=fmt_pars(cp), mode="grad_f", **sp)
    out["gradf_pois_m20_n1000"] = dict(kind="gradf", data="bench_pois", n=1000, spec=sp, cov_pars=cp, nll=r["nll"],
                                       grad=r["grad"], grad_f=rg["grad_f"])
    # predictions (latent means / variances, covariance with cond_all, response)
    X, y = data("bench_bern", 1000)
    npred = 40
    xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    xp[:5] = X[:5]
    cp = [1.0, 0.1]
    for pname, ptype, opts in [("pred_var_obs_only", "latent_order_obs_first_cond_obs_only", dict(predict_var="1")),
                               ("pred_cov_cond_all", "latent_order_obs_first_cond_all", dict(predict_cov="1")),
                               ("pred_resp_obs_only", "latent_order_obs_first_cond_obs_only",
                                dict(predict_var="1", predict_response="1"))]:
        sp = spec("bernoulli_logit", "exponential", 0.5, 20)
        # cond_all refuses prediction points on training coordinates (likelihoods.h: duplicates with '_cond_all')
        dup = ptype != "latent_order_obs_first_cond_all"
        xq = xp if dup else synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
        with open(os.path.join(HERE, "_pred_tmp.bin"), "wb") as f:
            f.write(np.array([npred], dtype=np.int32).tobytes())
            f.write(np.asfortranarray(xq).T.astype(np.float64).tobytes())
        try:
            r = run_ref(X, y, cov_pars=fmt_pars(cp), mode="predict", pred=os.path.join(HERE, "_pred_tmp.bin"),
                        vecchia_pred_type=ptype, **opts, **sp)
        finally:
            os.unlink(os.path.join(HERE, "_pred_tmp.bin"))
        c = dict(kind="pred", data="bench_bern", n=1000, npred=npred, dup5=dup, spec=sp, cov_pars=cp, vecchia_pred_type=ptype,
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
