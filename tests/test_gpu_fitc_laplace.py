"""GPU parity for the FITC approximation with a Laplace likelihood (gp_approx = "fitc",
likelihood = "bernoulli_logit") through the C ABI.

Reference: FindModePostRandEffCalcMLLFITC (likelihoods.h:3090-3235), CalcGradNegMargLikelihoodLaplaceApproxFITC
(:5397-5593), PredictLaplaceApproxFITC (:7157-7232) with CalcPredFITC_FSA (re_model_template.h:10600-10760),
CalcSigmaComps (:7341-7378). Fixtures: tests/golden/golden_fitc_laplace.json (the reference itself,
make_golden_fitc_laplace.py).

Tolerances: the Newton iterations run the reference's steps with the same stopping rule, so both land on
the same iterate up to rounding (fp64 MFMA GEMMs and explicit inverses vs Eigen's Cholesky solves): nll
1e-8, gradient 1e-6 (the north-star bound), predictions 1e-7; fits the same iteration count and
estimates to 1e-6.
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPBoostError, GPModel, synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_fitc_laplace.json")) as _f:
    GOLDEN = json.load(_f)
EVAL = [k for k in GOLDEN if k.startswith("fl_")]
FITS = [k for k in GOLDEN if k.startswith("fit_")]
PREDS = [k for k in GOLDEN if k.startswith("pred_")]


def _data(case):
    X = synthetic.bench_coords(case["n"])
    return X, synthetic.bench_bernoulli_y(X)


def _model(case, X):
    sp = case["spec"]
    return GPModel(gp_coords=X, cov_function=sp["cov_fct"], cov_fct_shape=float(sp.get("shape", 0.5)),
                   gp_approx="fitc", num_ind_points=int(sp["num_ind_points"]), likelihood="bernoulli_logit",
                   ind_points_selection=sp.get("ind_points_selection", "kmeans++"), seed=int(sp.get("seed", 0)))


@pytest.mark.parametrize("name", EVAL)
def test_fitc_laplace_matches_reference(name):
    case = GOLDEN[name]
    X, y = _data(case)
    gm = _model(case, X)
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= 1e-8 * abs(case["nll"]), (nll, case["nll"])
    np.testing.assert_allclose(g, case["grad"], rtol=1e-6, atol=1e-8 * abs(case["nll"]))
    # the objective without the gradient is the same number (a repeat from the zero mode)
    assert abs(gm.neg_log_likelihood(case["cov_pars"], y) - nll) <= 1e-12 * abs(nll)


def test_fitc_laplace_gradient_finite_differences():
    """The gradient is that of the returned objective (central differences in log-parameters)."""
    case = GOLDEN["fl_exp_n2000_m100"]
    X, y = _data(case)
    gm = _model(case, X)
    cp = np.array(case["cov_pars"])
    _, g, _ = gm.neg_log_likelihood_and_grad(cp, y)
    h = 1e-4
    for k in range(2):
        e = np.zeros(2)
        e[k] = h
        fp = gm.neg_log_likelihood(cp * np.exp(e), y)
        fm = gm.neg_log_likelihood(cp * np.exp(-e), y)
        fd = (fp - fm) / (2 * h)
        # the range enters through phi = 1 / rho: d/dlog rho = -d/dlog phi
        ref = g[k] if k == 0 else -g[k]
        assert abs(fd - ref) <= 1e-3 * max(1.0, abs(ref)), (k, fd, ref)


@pytest.mark.parametrize("name", FITS)
def test_fitc_laplace_fit_matches_reference(name):
    case = GOLDEN[name]
    X, y = _data(case)
    gm = _model(case, X)
    gm.fit(y)
    np.testing.assert_allclose(gm.get_init_cov_pars(), case["init_cov_pars"], rtol=1e-12)
    assert gm.get_num_optim_iter() == case["num_it"]
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-6)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-8 * abs(case["nll"])


def test_fitc_laplace_gradient_wrt_fixed_effects():
    """REModel::CalcGradient (CalcGradientF, re_model_template.h:3021-3043) with the FITC branch of
    CalcGradNegMargLikelihoodLaplaceApproxFITC calc_F_grad (likelihoods.h:5510-5531)."""
    case = GOLDEN["gradf_fl_exp_n2000_m80"]
    X, y = _data(case)
    fe = 0.3 * np.sin(3.0 * X[:, 0]) - 0.2
    gm = _model(case, X)
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y, fixed_effects=fe)
    assert abs(nll - case["nll"]) <= 1e-8 * abs(case["nll"])
    np.testing.assert_allclose(g, case["grad"], rtol=1e-6)
    gm.set_optim_params({"init_cov_pars": np.array(case["cov_pars"])})
    gf = gm.calc_gradient_f(fixed_effects=fe)
    ref = np.asarray(case["grad_f"])
    assert np.max(np.abs(gf - ref)) <= 1e-7 * max(1.0, np.max(np.abs(ref))), np.max(np.abs(gf - ref))


@pytest.mark.parametrize("name", PREDS)
def test_fitc_laplace_predict_matches_reference(name):
    case = GOLDEN[name]
    X, y = _data(case)
    npred = case["npred"]
    xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    if case["train_pts"]:
        k = case["train_pts"]
        xp[:k] = X[::max(1, case["n"] // k)][:k]
    gm = _model(case, X)
    want_cov = "cov" in case
    pred = gm.predict(y=y, gp_coords_pred=xp, cov_pars=case["cov_pars"], predict_var=not want_cov,
                      predict_cov_mat=want_cov, predict_response=case["response"])
    mu = np.asarray(case["mean"])
    np.testing.assert_allclose(pred["mu"], mu, rtol=1e-7, atol=1e-7 * np.abs(mu).max())
    if want_cov:
        c = np.asarray(case["cov"]).reshape(npred, npred)
        np.testing.assert_allclose(pred["cov"], c, rtol=1e-7, atol=1e-7 * np.abs(c).max())
    else:
        np.testing.assert_allclose(pred["var"], case["var"], rtol=1e-7, atol=1e-10)


def test_fitc_laplace_refusals():
    X = synthetic.bench_coords(500)
    with pytest.raises(GPBoostError, match="iterative"):
        GPModel(gp_coords=X, gp_approx="fitc", num_ind_points=20, likelihood="bernoulli_logit",
                matrix_inversion_method="iterative")
