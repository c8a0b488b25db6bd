"""GPU parity for likelihood 'gamma' (log link, shape parameter) through the C ABI: the dense Laplace path
(gp_approx = "none", DenseLaplace) and FITC (FitcLaplace) with the shape gradient and shape estimation, and
Vecchia-iterative evaluations with and without the shape gradient (stochastic diag((Sigma^-1 + W)^-1) from the
mode derivative, likelihoods.h:5126-5127). Reference: LogLikGamma / FirstDerivLogLikGamma / SecondDerivNegLogLikGamma and the
third derivative (likelihoods.h:8740, 9234, 9908, 10228), the shape gradient CalcGradNegLogLikAuxPars /
CalcSecondDerivLogLikFirstDerivInformationAuxPar (:10508-10524, :10856-10869) inside
CalcGradNegMargLikelihoodLaplaceApproxStable (:3379-3411), the normalizing constant (:8431-8449),
FindInitialAuxPars (:1116-1145) and PredictResponse (:7571-7584).

Fixtures: tests/golden/golden_gamma.json (the reference itself, make_golden_gamma.py), which reproduce the R
test's own values on its data (test_GPModel_non_Gaussian_data.R:2603-2625: nll 154.4561783, the lbfgs estimate
(1.0649277352, 0.2738906496) in 5 iterations). Tolerances as the dense Laplace suite (exact dense algebra): nll
1e-9, gradients 1e-7, fits 1e-6 with the reference's iteration count, predictions 1e-8; FITC nll 1e-8 / gradient
1e-6; Vecchia-iterative at cg_delta_conv = 1e-10: 1e-6 (north star).
"""
import json
import os

import numpy as np
import pytest

from conftest import lik_case_data

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_gamma.json")) as _f:
    GOLDEN = json.load(_f)


def _model(X, case):
    from gpboost_amd import GPModel
    sp = case["spec"]
    kw = dict(gp_coords=X, cov_function=sp["cov_fct"], cov_fct_shape=float(sp["shape"]), likelihood="gamma",
              gp_approx=sp["gp_approx"], seed=0)
    if sp["gp_approx"] == "fitc":
        kw["num_ind_points"] = int(sp["num_ind_points"])
    if sp["gp_approx"] == "vecchia":
        kw.update(num_neighbors=int(sp["num_neighbors"]), vecchia_ordering=sp["ordering"],
                  matrix_inversion_method="iterative")
    gm = GPModel(**kw)
    ex = case.get("extra", {})
    params = {}
    if "cg_delta_conv" in ex:
        params.update(cg_delta_conv=float(ex["cg_delta_conv"]), num_rand_vec_trace=int(ex["num_rand_vec_trace"]),
                      seed_rand_vec_trace=int(ex["seed_rand_vec_trace"]))
    if "aux_pars" in ex or "aux" in case:
        params["init_aux_pars"] = [float(ex.get("aux_pars", case.get("aux")))]
    params["estimate_aux_pars"] = bool(case.get("estimate_aux", False))
    gm.set_optim_params(params)
    return gm


@pytest.mark.parametrize("name", [k for k in GOLDEN if GOLDEN[k]["kind"] == "eval"])
def test_gamma_nll_grad_match_reference(name):
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    gm = _model(X, case)
    approx = case["spec"]["gp_approx"]
    tol_nll, tol_g = {"none": (1e-9, 1e-7), "fitc": (1e-8, 1e-6), "vecchia": (1e-6, 1e-6)}[approx]
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= tol_nll * abs(case["nll"]), (nll, case["nll"])
    ref = np.asarray(case["grad"])
    assert g.shape == ref.shape, (g, ref)
    np.testing.assert_allclose(g, ref, rtol=tol_g, atol=tol_g * np.abs(ref).max())
    if "r_expected_nll" in case:
        assert abs(nll - case["r_expected_nll"]) < 1e-5   # TOLERANCE_STRICT


@pytest.mark.parametrize("name", [k for k in GOLDEN if GOLDEN[k]["kind"] == "fit"])
def test_gamma_fit_matches_reference(name):
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    gm = _model(X, case)
    params = {}
    if "optimizer" in case["extra"]:
        params["optimizer_cov"] = case["extra"]["optimizer"]
    if "init_cov_pars" in case["extra"]:
        params["init_cov_pars"] = np.array([float(v) for v in case["extra"]["init_cov_pars"].split(",")])
    gm.fit(y, params=params)
    assert gm.get_num_optim_iter() == case["num_it"]
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-6)
    np.testing.assert_allclose(gm.get_aux_pars()[0], case["aux_pars"], rtol=1e-6)
    tol = 1e-9 if case["spec"]["gp_approx"] == "none" else 1e-8
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= tol * abs(case["nll"])
    if "r_expected_cov_pars" in case:
        assert np.sum(np.abs(gm.get_cov_pars() - case["r_expected_cov_pars"])) < 1e-5
        assert gm.get_num_optim_iter() == case["r_expected_num_it"]
    if "r_expected_aux_pars" in case:
        assert np.sum(np.abs(gm.get_aux_pars()[0] - case["r_expected_aux_pars"])) < 1e-5


@pytest.mark.parametrize("name", [k for k in GOLDEN if GOLDEN[k]["kind"] == "pred"])
def test_gamma_predict_matches_reference(name):
    from gpboost_amd import synthetic
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    npred = case["npred"]
    xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    gm = _model(X, case)
    want_cov = "cov" in case
    pred = gm.predict(y=y, gp_coords_pred=xp, cov_pars=case["cov_pars"], predict_var=not want_cov,
                      predict_cov_mat=want_cov, predict_response=case["response"])
    mu = np.asarray(case["mean"])
    np.testing.assert_allclose(pred["mu"], mu, rtol=1e-8, atol=1e-8 * np.abs(mu).max())
    if want_cov:
        c = np.asarray(case["cov"]).reshape(npred, npred)
        np.testing.assert_allclose(pred["cov"], c, rtol=1e-8, atol=1e-8 * np.abs(c).max())
    else:
        np.testing.assert_allclose(pred["var"], case["var"], rtol=1e-8, atol=1e-11)


def test_gamma_checks_and_refusals():
    from gpboost_amd import GPModel, GPBoostError, synthetic
    X, y = synthetic.rtest_gamma_y(100)
    gm = GPModel(gp_coords=X, likelihood="gamma", cov_function="exponential")
    with pytest.raises(GPBoostError, match="y > 0"):
        gm.neg_log_likelihood([1.0, 0.2], np.where(np.arange(100) == 7, 0.0, y))
    assert gm.get_aux_pars()[1] == "shape"
    # repeated coordinates: the shape gradient of the Vecchia path is refused (unique-location form)
    Xd = np.vstack([X[:50], X[:50]])
    gv = GPModel(gp_coords=Xd, likelihood="gamma", cov_function="exponential", gp_approx="vecchia", num_neighbors=10,
                 matrix_inversion_method="iterative")
    with pytest.raises(GPBoostError, match="estimate_aux_pars"):
        gv.fit(y)


def test_gamma_fixed_covariance_parameters_r_test():
    """estimate_cov_par_index with likelihood 'gamma' (test_GPModel_non_Gaussian_data.R:2646-2676): lbfgs with both
    covariance parameters fixed at (1, mean(dist) / 3) estimates the shape alone (0.9902641, TOLERANCE_STRICT);
    with one of them fixed the fixed one keeps its initial value (dense and FITC)."""
    from gpboost_amd import GPModel, synthetic
    X, y = synthetic.rtest_gamma_y(100)
    D = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    init = np.array([1.0, D[np.triu_indices(100, 1)].mean() / 3])
    gm = GPModel(gp_coords=X, cov_function="exponential", likelihood="gamma")
    gm.fit(y, params={"optimizer_cov": "lbfgs", "init_cov_pars": init, "init_aux_pars": [1.0],
                      "estimate_aux_pars": True, "estimate_cov_par_index": [0, 0]})
    assert np.sum(np.abs(gm.get_cov_pars() - [1.0, 0.1786481])) < 1e-5
    assert abs(gm.get_aux_pars()[0][0] - 0.9902641) < 1e-5
    for approx in ("none", "fitc"):
        for idx in ([1, 0], [0, 1]):
            kw = dict(num_ind_points=50) if approx == "fitc" else {}
            gm = GPModel(gp_coords=X, cov_function="exponential", likelihood="gamma", gp_approx=approx, **kw)
            gm.fit(y, params={"optimizer_cov": "lbfgs", "init_cov_pars": init, "init_aux_pars": [2.0],
                              "estimate_aux_pars": True, "estimate_cov_par_index": idx})
            k = idx.index(0)
            assert abs(gm.get_cov_pars()[k] - init[k]) < 1e-5


def test_gamma_gradient_descent_r_test():
    """gradient_descent (Nesterov) for a Laplace model with the shape estimated (test_GPModel_non_Gaussian_data.R:
    2636-2645): (1.0323441289, 0.2898716638), shape 0.9413081183, 26 iterations (TOLERANCE_STRICT 1e-5)."""
    from gpboost_amd import GPModel, synthetic
    X, y = synthetic.rtest_gamma_y(100)
    D = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    init = np.array([1.0, D[np.triu_indices(100, 1)].mean() / 3])
    gm = GPModel(gp_coords=X, cov_function="exponential", likelihood="gamma")
    gm.fit(y, params={"optimizer_cov": "gradient_descent", "init_cov_pars": init, "init_aux_pars": [1.0],
                      "estimate_aux_pars": True})
    assert np.sum(np.abs(gm.get_cov_pars() - [1.0323441289, 0.2898716638])) < 1e-5, gm.get_cov_pars()
    assert abs(gm.get_aux_pars()[0][0] - 0.9413081183) < 1e-5, gm.get_aux_pars()
    assert gm.get_num_optim_iter() == 26
