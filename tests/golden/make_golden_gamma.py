#!/usr/bin/env python3
"""Reference fixtures for likelihood 'gamma' (log link, shape parameter; likelihoods.h LogLikGamma :8740,
FirstDerivLogLikGamma :9234, SecondDerivNegLogLikGamma :9908, third derivative :10228, shape gradient
:10508-10524 / :10856-10869, normalizing constant :8431-8449, FindInitialAuxPars :1116-1145, PredictResponse
:7571-7584), from the reference itself (oracle/_ref/ref_harness built from /root/reference by oracle/Makefile):

    make -C oracle ref && python3 tests/golden/make_golden_gamma.py

Dense (gp_approx = "none") evaluations with the shape gradient, fits with and without shape estimation,
predictions; FITC and Vecchia-iterative evaluations at a fixed shape. Inputs from gpboost_amd/synthetic.py;
outputs are the reference's.
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
from make_golden_latent_lik import data  # noqa: E402

OUT = os.path.join(HERE, "golden_gamma.json")
AUX_ARGS = dict(num_rand_vec_trace="50")   # routes the harness through SetOptimConfig (estimate_aux honoured)


def eval_case(kind, n, cp, aux, estimate_aux, **sp):
    X, y = data(kind, n)
    spec = dict(likelihood="gamma", cov_fct=sp.get("cov_fct", "exponential"), shape=str(sp.get("shape", 0.5)),
                gp_approx=sp.get("gp_approx", "none"), matrix_inversion_method=sp.get("mim", "cholesky"))
    for k in ("num_ind_points", "num_neighbors", "ordering"):
        if k in sp:
            spec[k] = sp[k]
    extra = dict(AUX_ARGS, estimate_aux=str(int(estimate_aux)), aux_pars=repr(float(aux)))
    if "cg_delta_conv" in sp:
        extra.update(cg_delta_conv=repr(sp["cg_delta_conv"]), num_rand_vec_trace=str(sp.get("t", 50)),
                     seed_rand_vec_trace="1")
    r = run_ref(X, y, cov_pars=fmt_pars(cp), mode="eval", **spec, **extra)
    return dict(kind="eval", data=kind, n=n, cov_pars=list(cp), aux=aux, estimate_aux=estimate_aux, spec=spec,
                extra=extra, nll=r["nll"], grad=r["grad"])


def fit_case(kind, n, estimate_aux, init=None, aux=None, optimizer=None, **sp):
    X, y = data(kind, n)
    spec = dict(likelihood="gamma", cov_fct=sp.get("cov_fct", "exponential"), shape=str(sp.get("shape", 0.5)),
                gp_approx=sp.get("gp_approx", "none"))
    if "num_ind_points" in sp:
        spec["num_ind_points"] = sp["num_ind_points"]
    extra = dict(estimate_aux=str(int(estimate_aux)))
    if init is not None:
        extra["init_cov_pars"] = fmt_pars(init)
    if aux is not None:
        extra["aux_pars"] = repr(float(aux))
    if optimizer is not None:
        extra["optimizer"] = optimizer
    r = run_ref(X, y, mode="fit", **spec, **extra)
    out = dict(kind="fit", data=kind, n=n, estimate_aux=estimate_aux, spec=spec, extra=extra,
               **{k: r[k] for k in ("init_cov_pars", "cov_pars", "nll", "num_it")})
    if "aux_pars" in r:
        out["aux_pars"] = r["aux_pars"]
    return out


def pred_case(kind, n, npred, cp, aux, cov=False, response=False):
    X, y = data(kind, n)
    Xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([npred], dtype=np.int32).tobytes())
        f.write(np.asfortranarray(Xp).T.astype(np.float64).tobytes())
        ppath = f.name
    spec = dict(likelihood="gamma", cov_fct="exponential", shape="0.5", gp_approx="none")
    extra = {"predict_cov": "1"} if cov else {"predict_var": "1"}
    if response:
        extra["predict_response"] = "1"
    try:
        r = run_ref(X, y, cov_pars=fmt_pars(cp), mode="predict", pred=ppath, aux_pars=repr(float(aux)), **spec, **extra)
    finally:
        os.unlink(ppath)
    out = dict(kind="pred", data=kind, n=n, npred=npred, cov_pars=list(cp), aux=aux, spec=spec, response=response,
               mean=r["mean"])
    out["cov" if cov else "var"] = r["cov" if cov else "var"]
    return out


def main():
    Xr, _ = synthetic.rtest_gamma_y(100)
    D = np.sqrt(((Xr[:, None, :] - Xr[None, :, :]) ** 2).sum(-1))
    mean_dist = D[np.triu_indices(100, 1)].mean()
    cases = {
        "ev_rtest_dense": eval_case("rtest_gamma", 100, (0.9, 0.2), 1.0, False),
        "ev_rtest_dense_shape_grad": eval_case("rtest_gamma", 100, (0.9, 0.2), 1.0, True),
        "ev_bench_dense_matern15_shape2": eval_case("bench_gamma", 800, (0.7, 0.15), 2.0, True, cov_fct="matern",
                                                    shape=1.5),
        "ev_bench_dense_exp_shape07": eval_case("bench_gamma", 600, (1.1, 0.1), 0.7, True),
        "ev_bench_fitc": eval_case("bench_gamma", 1500, (0.7, 0.15), 2.0, False, gp_approx="fitc", num_ind_points=60),
        "ev_bench_fitc_shape_grad": eval_case("bench_gamma", 1500, (0.7, 0.15), 2.0, True, gp_approx="fitc",
                                              num_ind_points=60),
        "fit_bench_fitc_shape": fit_case("bench_gamma", 1000, True, gp_approx="fitc", num_ind_points=50),
        "ev_bench_vecchia_tight": eval_case("bench_gamma", 2000, (0.7, 0.15), 2.0, False, gp_approx="vecchia",
                                            mim="iterative", num_neighbors=20, ordering="random", cg_delta_conv=1e-10),
        "ev_bench_vecchia_tight_shape_grad": eval_case("bench_gamma", 2000, (0.7, 0.15), 2.0, True, gp_approx="vecchia",
                                                       mim="iterative", num_neighbors=20, ordering="random",
                                                       cg_delta_conv=1e-10),
        # test_GPModel_non_Gaussian_data.R:2605-2614: lbfgs, shape fixed at 1, init (1, mean(dist) / 3)
        "fit_rtest_fixed_shape": fit_case("rtest_gamma", 100, False, init=(1.0, mean_dist / 3), aux=1.0),
        "fit_bench_shape": fit_case("bench_gamma", 500, True),
        # :2626-2635: nelder_mead with the shape estimated, init (1, mean(dist) / 3), shape 1
        "fit_rtest_nm_shape": fit_case("rtest_gamma", 100, True, init=(1.0, mean_dist / 3), aux=1.0,
                                       optimizer="nelder_mead"),
        "pred_rtest_cov": pred_case("rtest_gamma", 100, 3, (1.0, 0.3), 1.0, cov=True),
        "pred_bench_resp": pred_case("bench_gamma", 600, 100, (0.7, 0.15), 2.0, response=True),
    }
    cases["ev_rtest_dense"]["r_expected_nll"] = 154.4561783                                  # :2624-2625
    cases["fit_rtest_fixed_shape"]["r_expected_cov_pars"] = [1.0649277352, 0.2738906496]     # :2613
    cases["fit_rtest_fixed_shape"]["r_expected_num_it"] = 5                                  # :2614
    cases["fit_rtest_nm_shape"]["r_expected_cov_pars"] = [1.0445949478, 0.2971884204]        # :2631-2635
    cases["fit_rtest_nm_shape"]["r_expected_aux_pars"] = [0.9400943304]
    cases["fit_rtest_nm_shape"]["r_expected_num_it"] = 115
    for k, v in cases.items():
        print(k, v.get("nll"), v.get("grad", v.get("cov_pars")), v.get("num_it"), v.get("aux_pars"), file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f)


if __name__ == "__main__":
    main()
