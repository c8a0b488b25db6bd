"""GPU parity for the Laplace approximation without a GP approximation (gp_approx = "none", the reference's
default for non-Gaussian likelihoods), through the C ABI: DenseLaplace (csrc/dense_laplace.h) against
FindModePostRandEffCalcMLLStable, CalcGradNegMargLikelihoodLaplaceApproxStable and
PredictLaplaceApproxStable (likelihoods.h:1843-1960, 3261-3413, 5610-5676).

Fixtures: tests/golden/golden_dense_laplace.json (the reference itself, make_golden_dense_laplace.py) for
bernoulli_logit / bernoulli_probit / poisson and four covariance functions, plus the R tests' hard-coded
values on their own data (test_GPModel_non_Gaussian_data.R:1196 probit 67.18342059, :2410 poisson
195.03708036, tolerance 1e-5 there). Both sides are exact dense algebra, so the nll must agree to 1e-9
relative, gradients to 1e-7, fits with the reference's iteration count to 1e-6, predictions to 1e-8.
"""
import json
import os

import numpy as np
import pytest

from conftest import lik_case_data

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_dense_laplace.json")) as _f:
    GOLDEN = json.load(_f)


def _of(kind):
    return [k for k in GOLDEN if GOLDEN[k]["kind"] == kind]


def _model(X, case):
    from gpboost_amd import GPModel
    sp = case["spec"]
    return GPModel(gp_coords=X, cov_function=sp["cov_fct"], cov_fct_shape=float(sp["shape"]), likelihood=sp["likelihood"])


@pytest.mark.parametrize("name", _of("eval"))
def test_dense_laplace_nll_grad_match_reference(name):
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    gm = _model(X, case)
    nll = gm.neg_log_likelihood(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= 1e-9 * abs(case["nll"]), (nll, case["nll"])
    nll2, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert abs(nll2 - case["nll"]) <= 1e-9 * abs(case["nll"])
    ref = np.asarray(case["grad"])
    np.testing.assert_allclose(g, ref, rtol=1e-7, atol=1e-9 * abs(case["nll"]))
    if "r_expected_nll" in case:   # the R test's own value (TOLERANCE_STRICT = 1e-5)
        assert abs(nll - case["r_expected_nll"]) < 1e-5


@pytest.mark.parametrize("name", _of("fit"))
def test_dense_laplace_fit_matches_reference(name):
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    gm = _model(X, case)
    gm.fit(y)
    np.testing.assert_allclose(gm.get_init_cov_pars(), case["init_cov_pars"], rtol=1e-12)
    assert gm.get_num_optim_iter() == case["num_it"]
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-6)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-9 * abs(case["nll"])


@pytest.mark.parametrize("name", _of("gradf"))
def test_dense_laplace_gradient_wrt_fixed_effects(name):
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    fe = 0.3 * np.sin(3.0 * X[:, 0]) - 0.2
    gm = _model(X, case)
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y, fixed_effects=fe)
    assert abs(nll - case["nll"]) <= 1e-9 * abs(case["nll"])
    np.testing.assert_allclose(g, case["grad"], rtol=1e-7)
    gm.set_optim_params({"init_cov_pars": np.array(case["cov_pars"])})
    gf = gm.calc_gradient_f(fixed_effects=fe)
    ref = np.asarray(case["grad_f"])
    assert np.max(np.abs(gf - ref)) <= 1e-8 * max(1.0, np.max(np.abs(ref))), np.max(np.abs(gf - ref))


@pytest.mark.parametrize("name", _of("pred"))
def test_dense_laplace_predict_matches_reference(name):
    from gpboost_amd import synthetic
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    npred = case["npred"]
    xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    xp[: min(5, npred)] = X[: min(5, npred)]
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


def test_dense_laplace_refusals_and_switch():
    from gpboost_amd import GPModel, GPBoostError, synthetic
    X, y = synthetic.rtest_bernoulli_probit_y(100)
    with pytest.raises(GPBoostError, match="iterative"):
        GPModel(gp_coords=X, likelihood="bernoulli_probit", cov_function="exponential", matrix_inversion_method="iterative")
    with pytest.raises(GPBoostError, match="duplicate"):
        GPModel(gp_coords=np.vstack([X[:50], X[:50]]), likelihood="bernoulli_probit")
    # likelihood switch gaussian -> probit on a dense model (GPB_SetLikelihood, the R package's set_likelihood;
    # re_model.cpp:142-147) reaches the same value
    from gpboost_amd.basic import _safe_call, c_str, lib
    gm = GPModel(gp_coords=X, likelihood="gaussian", cov_function="exponential")
    _safe_call(lib().GPB_SetLikelihood(gm.handle, c_str("bernoulli_probit")))
    gm.num_cov_pars = 2
    nll = gm.neg_log_likelihood([1.0, 0.2], y)
    assert abs(nll - GOLDEN["ev_rtest_probit"]["nll"]) <= 1e-9 * abs(nll)


def test_dense_laplace_probit_r_test_optimizers():
    """test_GPModel_non_Gaussian_data.R:105-165 on its own data (probit GP, gp_approx = "none", cholesky): gradient
    descent without acceleration (parameter criterion) 40 iterations, with Nesterov (lr 0.01) 26, Nelder-Mead 6, each
    at TOLERANCE_STRICT 1e-5; predictions of the lr-0.01 gradient-descent fit (means and covariance, 1e-5)."""
    from gpboost_amd import GPModel, synthetic
    X, y = synthetic.rtest_bernoulli_probit_y(100, init_c=0.2341)
    D = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    init = np.array([1.0, D[np.triu_indices(100, 1)].mean() / 3])

    def fit(params):
        gm = GPModel(gp_coords=X, cov_function="exponential", likelihood="bernoulli_probit",
                     matrix_inversion_method="cholesky")
        gm.fit(y, params=dict(params, init_cov_pars=init))
        return gm

    gm = fit(dict(optimizer_cov="gradient_descent", lr_cov=0.1, use_nesterov_acc=False,
                  convergence_criterion="relative_change_in_parameters"))
    assert np.sum(np.abs(gm.get_cov_pars() - [0.9419234, 0.1866877])) < 1e-5
    assert abs(gm.get_current_neg_log_likelihood() - 63.61263619) < 1e-5
    assert gm.get_num_optim_iter() == 40
    gm = fit(dict(optimizer_cov="gradient_descent", lr_cov=0.01, use_nesterov_acc=True, acc_rate_cov=0.5))
    assert np.sum(np.abs(gm.get_cov_pars() - [0.9646422, 0.1844797])) < 1e-5
    assert gm.get_num_optim_iter() == 26
    gm = fit(dict(optimizer_cov="nelder_mead", delta_rel_conv=1e-6))
    assert np.sum(np.abs(gm.get_cov_pars() - [0.9998047, 0.1855072])) < 1e-5
    assert gm.get_num_optim_iter() == 6
    gm = fit(dict(optimizer_cov="gradient_descent", lr_cov=0.01, use_nesterov_acc=False))
    xp = np.array([[0.1, 0.9], [0.11, 0.91], [0.7, 0.55]])
    pred = gm.predict(y=y, gp_coords_pred=xp, predict_cov_mat=True, predict_response=False)
    assert np.sum(np.abs(pred["mu"] - [-0.6595663, -0.6638940, 0.4997690])) < 1e-5
    cov = [0.6482224576, 0.5765285950, -0.0001030520, 0.5765285950, 0.6478191338, -0.0001163496, -0.0001030520,
           -0.0001163496, 0.4435551436]
    assert np.sum(np.abs(np.asarray(pred["cov"]).T.reshape(-1) - cov)) < 1e-5


def test_dense_laplace_poisson_r_test():
    """test_GPModel_non_Gaussian_data.R:2385-2410 on its own data (Poisson GP, gp_approx = "none"): gradient descent
    with Nesterov (DEFAULT_OPTIM_PARAMS, lr 0.1) from (1, mean(dist) / 3): (1.1853922, 0.1500197) in 6 iterations
    (1e-5); latent predictive means (1e-3) and covariance (1e-5); response means / variances (1e-3)."""
    from gpboost_amd import GPModel, synthetic
    X, y = synthetic.rtest_poisson_y(100)
    D = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    init = np.array([1.0, D[np.triu_indices(100, 1)].mean() / 3])
    gm = GPModel(gp_coords=X, cov_function="exponential", likelihood="poisson")
    gm.fit(y, params=dict(optimizer_cov="gradient_descent", use_nesterov_acc=True, lr_cov=0.1, maxit=1000,
                          acc_rate_cov=0.5, init_cov_pars=init))
    assert np.sum(np.abs(gm.get_cov_pars() - [1.1853922, 0.1500197])) < 1e-5, gm.get_cov_pars()
    assert gm.get_num_optim_iter() == 6
    xp = np.array([[0.1, 0.9], [0.11, 0.91], [0.7, 0.55]])
    pred = gm.predict(y=y, gp_coords_pred=xp, predict_cov_mat=True, predict_response=False)
    assert np.sum(np.abs(pred["mu"] - [0.4329068, 0.4042531, 0.6833738])) < 1e-3
    cov = [6.550626e-01, 5.553938e-01, -8.406290e-06, 5.553938e-01, 6.631295e-01, -7.658261e-06, -8.406290e-06,
           -7.658261e-06, 4.170417e-01]
    assert np.sum(np.abs(np.asarray(pred["cov"]).T.reshape(-1) - cov)) < 1e-5
    pred = gm.predict(y=y, gp_coords_pred=xp, predict_var=True, predict_response=True)
    assert np.sum(np.abs(pred["mu"] - [2.139213, 2.087188, 2.439748])) < 1e-3
    assert np.sum(np.abs(pred["var"] - [6.373433, 6.185895, 5.519896])) < 1e-3


def test_dense_laplace_logit_r_test():
    """test_GPModel_non_Gaussian_data.R:2298-2328 on its own data (bernoulli_logit GP, gp_approx = "none"): Nesterov
    gradient descent (lr 0.01) from (1, mean(dist) / 3): (1.4300136, 0.1891952) in 85 iterations (1e-5); predictive
    means (1e-5) and covariance (1e-3); response probabilities and variances (adaptive Gauss-Hermite, 1e-5); nll at
    (0.9, 0.2) 66.299571 (1e-5)."""
    from gpboost_amd import GPModel, synthetic
    X, eps = synthetic._rtest_field(100)
    y = (synthetic.sim_rand_unif(100, 0.2341) < 1. / (1. + np.exp(-eps))).astype(np.float64)
    D = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    init = np.array([1.0, D[np.triu_indices(100, 1)].mean() / 3])
    gm = GPModel(gp_coords=X, cov_function="exponential", likelihood="bernoulli_logit")
    gm.fit(y, params=dict(optimizer_cov="gradient_descent", use_nesterov_acc=True, lr_cov=0.01, maxit=1000,
                          acc_rate_cov=0.5, init_cov_pars=init))
    assert np.sum(np.abs(gm.get_cov_pars() - [1.4300136, 0.1891952])) < 1e-5, gm.get_cov_pars()
    assert gm.get_num_optim_iter() == 85
    xp = np.array([[0.1, 0.9], [0.11, 0.91], [0.7, 0.55]])
    pred = gm.predict(y=y, gp_coords_pred=xp, predict_cov_mat=True, predict_response=False)
    assert np.sum(np.abs(pred["mu"] - [-0.7792960, -0.7876208, 0.5476390])) < 1e-5
    cov = [1.024266883e+00, 9.215203622e-01, 5.561463409e-05, 9.215203622e-01, 1.022897212e+00, 2.028646043e-05,
           5.561463409e-05, 2.028646043e-05, 7.395745025e-01]
    assert np.sum(np.abs(np.asarray(pred["cov"]).T.reshape(-1) - cov)) < 1e-3
    pred = gm.predict(y=y, gp_coords_pred=xp, predict_var=True, predict_response=True)
    mu = np.array([0.3442815, 0.3426873, 0.6159933])
    assert np.sum(np.abs(pred["mu"] - mu)) < 1e-5
    assert np.sum(np.abs(pred["var"] - mu * (1 - mu))) < 1e-5
    assert abs(gm.neg_log_likelihood([0.9, 0.2], y) - 66.299571) < 1e-5
