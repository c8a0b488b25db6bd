#!/usr/bin/env python3
"""Reference fixtures for the Laplace likelihoods bernoulli_probit and poisson, from the reference itself
(oracle/_ref/ref_harness built from /root/reference by oracle/Makefile):

    make -C oracle ref && python3 tests/golden/make_golden_latent_lik.py

* Vecchia + iterative methods (gp_approx = "vecchia", VADU preconditioner, probes from
  seed_rand_vec_trace): nll and gradient at a tight (1e-10) and the default (1e-2) cg_delta_conv;
  the likelihood enters through FindModePostRandEffCalcMLLVecchia's derivatives
  (likelihoods.h CalcFirstDerivLogLik / CalcSecondNegDerivLogLik / CalcThirdDerivLogLik, poisson
  normalizing constant CalculateAuxQuantLogNormalizingConstant).
* FITC (gp_approx = "fitc", cholesky): nll + gradient (FindModePostRandEffCalcMLLFITC,
  CalcGradNegMargLikelihoodLaplaceApproxFITC), a fit, the gradient wrt fixed effects and latent /
  response predictions (PredictResponse likelihoods.h:7526-7569).
* The R tests' own data (n = 100) at the parameters their hard-coded nll values are quoted on
  (test_GPModel_non_Gaussian_data.R:1196 probit 67.18342059 dense,
  :2410 poisson 195.03708036 dense), evaluated here by the reference's dense path as an anchor
  for the data generators; the GPU tests compare with these numbers at the R tests' tolerance.

Inputs are regenerated from the portable LCG generators (gpboost_amd/synthetic.py).
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, fmt_pars, run_ref  # noqa: E402

sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from gpboost_amd import synthetic  # noqa: E402

OUT = os.path.join(HERE, "golden_latent_lik.json")


def data(kind, n):
    if kind == "rtest_probit":
        return synthetic.rtest_bernoulli_probit_y(n)
    if kind == "rtest_poisson":
        return synthetic.rtest_poisson_y(n)
    if kind == "rtest_gamma":
        return synthetic.rtest_gamma_y(n)
    X = synthetic.bench_coords(n)
    if kind == "bench_gamma":
        return X, synthetic.bench_gamma_y(X)
    return X, (synthetic.bench_poisson_y(X) if kind == "bench_pois" else synthetic.bench_bernoulli_y(X))


def vecchia_case(kind, n, lik, cov_fct, shape, m, cp, dc, t, seed, ordering="random", fe=None):
    X, y = data(kind, n)
    opts = dict(cov_fct=cov_fct, shape=shape, num_neighbors=m, ordering=ordering, likelihood=lik,
                matrix_inversion_method="iterative", cov_pars=fmt_pars(cp), cg_delta_conv=repr(dc),
                num_rand_vec_trace=t, seed_rand_vec_trace=seed, gp_approx="vecchia")
    r = run_ref(X, y, fe=fe, **opts)
    return dict(kind="vecchia", data=kind, n=n, likelihood=lik, cov_fct=cov_fct, shape=shape, num_neighbors=m,
                ordering=ordering, cov_pars=list(cp), cg_delta_conv=dc, num_rand_vec_trace=t,
                seed_rand_vec_trace=seed, nll=r["nll"], grad=r["grad"])


def fitc_spec(lik, m, cov_fct="exponential", shape=0.5, sel="kmeans++", seed=0):
    return dict(cov_fct=cov_fct, shape=str(shape), gp_approx="fitc", num_ind_points=m, ind_points_selection=sel,
                seed=seed, likelihood=lik)


def fitc_case(kind, n, lik, m, cp, **kw):
    X, y = data(kind, n)
    spec = fitc_spec(lik, m, **kw)
    r = run_ref(X, y, cov_pars=fmt_pars(cp), mode="eval", **spec)
    return dict(kind="fitc", data=kind, n=n, m=m, likelihood=lik, cov_pars=list(cp), spec=spec, nll=r["nll"],
                grad=r["grad"], ind_points=r["ind_points"])


def fitc_fit_case(kind, n, lik, m, **kw):
    X, y = data(kind, n)
    spec = fitc_spec(lik, m, **kw)
    r = run_ref(X, y, mode="fit", **spec)
    return dict(kind="fitc_fit", data=kind, n=n, m=m, likelihood=lik, spec=spec,
                **{k: r[k] for k in r if k not in ("ok", "n", "d")})


def fitc_gradf_case(kind, n, lik, m, cp, **kw):
    X, y = data(kind, n)
    fe = 0.3 * np.sin(3.0 * X[:, 0]) - 0.2
    spec = fitc_spec(lik, m, **kw)
    r = run_ref(X, y, fe=fe, cov_pars=fmt_pars(cp), mode="grad_f", **spec)
    ev = run_ref(X, y, fe=fe, cov_pars=fmt_pars(cp), mode="eval", **spec)
    return dict(kind="fitc_gradf", data=kind, n=n, m=m, likelihood=lik, cov_pars=list(cp), spec=spec,
                grad_f=r["grad_f"], nll=ev["nll"], grad=ev["grad"], ind_points=ev["ind_points"])


def fitc_pred_case(kind, n, lik, m, npred, cp, cov=False, response=False, **kw):
    X, y = data(kind, n)
    Xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([npred], dtype=np.int32).tobytes())
        f.write(np.asfortranarray(Xp).T.astype(np.float64).tobytes())
        ppath = f.name
    spec = fitc_spec(lik, m, **kw)
    extra = {"predict_cov": "1"} if cov else {"predict_var": "1"}
    if response:
        extra["predict_response"] = "1"
    try:
        r = run_ref(X, y, cov_pars=fmt_pars(cp), mode="predict", pred=ppath, **spec, **extra)
    finally:
        os.unlink(ppath)
    out = dict(kind="fitc_pred", data=kind, n=n, m=m, likelihood=lik, npred=npred, cov_pars=list(cp), spec=spec,
               response=response, mean=r["mean"])
    out["cov" if cov else "var"] = r["cov" if cov else "var"]
    return out


def rtest_dense(kind, lik, cp, fe=None):
    X, y = data(kind, 100)
    r = run_ref(X, y, fe=fe, cov_fct="exponential", gp_approx="none", likelihood=lik, matrix_inversion_method="cholesky",
                cov_pars=fmt_pars(cp), mode="eval")
    return dict(kind="rtest_dense", data=kind, n=100, likelihood=lik, cov_pars=list(cp), nll=r["nll"], grad=r["grad"])


def main():
    pr, po = "bernoulli_probit", "poisson"
    cases = {
        "vp_probit_m30_exp_tight": vecchia_case("bench_bern", 2000, pr, "exponential", 0.5, 30, [1.0, 0.1], 1e-10, 50, 1),
        "vp_probit_m30_exp_default": vecchia_case("bench_bern", 2000, pr, "exponential", 0.5, 30, [1.0, 0.1], 1e-2, 50, 1),
        "vp_probit_m16_matern15": vecchia_case("bench_bern", 2000, pr, "matern", 1.5, 16, [0.7, 0.12], 1e-8, 30, 4),
        "vp_pois_m30_exp_tight": vecchia_case("bench_pois", 2000, po, "exponential", 0.5, 30, [0.8, 0.1], 1e-10, 50, 1),
        "vp_pois_m30_exp_default": vecchia_case("bench_pois", 2000, po, "exponential", 0.5, 30, [0.8, 0.1], 1e-2, 50, 1),
        "vp_pois_m20_matern25": vecchia_case("bench_pois", 3000, po, "matern", 2.5, 20, [0.5, 0.07], 1e-8, 40, 2),
        "vp_rtest_probit_m30": vecchia_case("rtest_probit", 100, pr, "exponential", 0.5, 30, [1.0, 0.2], 1e-10, 50, 1),
        "vp_rtest_pois_m30": vecchia_case("rtest_poisson", 100, po, "exponential", 0.5, 30, [0.9, 0.2], 1e-10, 50, 1),
        "fp_probit_exp_n2000_m100": fitc_case("bench_bern", 2000, pr, 100, (1.0, 0.1)),
        "fp_probit_matern15_n3000_m80": fitc_case("bench_bern", 3000, pr, 80, (1.3, 0.15), cov_fct="matern", shape=1.5),
        "fp_pois_exp_n2000_m100": fitc_case("bench_pois", 2000, po, 100, (0.8, 0.1)),
        "fp_pois_gauss_n2500_m60_random": fitc_case("bench_pois", 2500, po, 60, (0.6, 0.2), cov_fct="gaussian",
                                                    shape=0.0, sel="random", seed=3),
        # all n = 100 points as inducing points: FITC reproduces the dense R goldens up to the 1e-6 jitter
        "fp_rtest_probit_mall": fitc_case("rtest_probit", 100, pr, 100, (1.0, 0.2)),
        "fp_rtest_pois_mall": fitc_case("rtest_poisson", 100, po, 100, (0.9, 0.2)),
        "fitfp_probit_exp_n2000_m50": fitc_fit_case("bench_bern", 2000, pr, 50),
        "fitfp_pois_exp_n2000_m50": fitc_fit_case("bench_pois", 2000, po, 50),
        "gradffp_pois_exp_n2000_m80": fitc_gradf_case("bench_pois", 2000, po, 80, (0.8, 0.1)),
        "gradffp_probit_exp_n2000_m80": fitc_gradf_case("bench_bern", 2000, pr, 80, (1.0, 0.1)),
        "predfp_probit_resp": fitc_pred_case("bench_bern", 2000, pr, 60, 300, (1.0, 0.1), response=True),
        "predfp_pois_resp": fitc_pred_case("bench_pois", 2000, po, 60, 300, (0.8, 0.1), response=True),
        "predfp_pois_cov": fitc_pred_case("bench_pois", 1500, po, 60, 100, (0.8, 0.1), cov=True),
    }
    # gp_model$neg_log_likelihood(cov_pars, y) passes no fixed effects (R-package/R/GPModel.R:1126)
    cases["rtest_dense_probit"] = rtest_dense("rtest_probit", pr, [1.0, 0.2])
    cases["rtest_dense_probit"]["r_expected_nll"] = 67.18342059      # test_GPModel_non_Gaussian_data.R:1196
    cases["rtest_dense_pois"] = rtest_dense("rtest_poisson", po, [0.9, 0.2])
    cases["rtest_dense_pois"]["r_expected_nll"] = 195.03708036       # :2410
    for k, v in cases.items():
        print(k, v.get("nll"), v.get("grad", v.get("cov_pars")), file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f)


if __name__ == "__main__":
    main()
