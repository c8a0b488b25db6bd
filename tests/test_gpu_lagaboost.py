"""GPU parity for the GPBoost-algorithm entry points (LaGaBoost = BASELINE
config 5's name): likelihood evaluations with fixed effects F (the boosting score as an offset of
the location parameter), the gradient wrt F that the boosting objective uses as its pseudo-residual
(REModel::CalcGradient -> CalcGradientF, re_model_template.h:3021-3043; the Laplace-Vecchia form
likelihoods.h:5337-5367), and a covariance fit with the score as offset (REModel::OptimCovPar(nullptr,
score), regression_objective.hpp:178). Fixtures: tests/golden/golden_lagaboost.json
(make_golden_lagaboost.py, the reference itself).

Tolerances: exact Gaussian closed forms 1e-9; latent evaluations at cg_delta_conv = 1e-10 with the
reference's probe streams at the north-star 1e-6; the latent fit (cg_delta_conv = 1e-6) at 1e-4 like
the other latent fits (test_gpu_optim.py).
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPModel, synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
RTOL = 1e-6


@pytest.fixture(scope="module")
def golden_lb():
    with open(os.path.join(HERE, "golden", "golden_lagaboost.json")) as f:
        return json.load(f)


def _offset(X):
    return 0.5 * np.sin(3 * X[:, 0]) - 0.3 * X[:, 1]


def _bern(n, cg=1e-10):
    X = synthetic.bench_coords(n)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", likelihood="bernoulli_logit",
                 num_neighbors=30, vecchia_ordering="random", seed=0)
    gm.set_optim_params({"cg_delta_conv": cg})
    return X, gm


def _close(a, b, rtol=RTOL):
    a, b = np.asarray(a, float), np.asarray(b, float)
    scale = max(np.max(np.abs(b)), 1.0)
    return np.max(np.abs(a - b)) <= rtol * scale


def test_bernoulli_with_offset_matches_reference(golden_lb):
    case = golden_lb["bernoulli_offset"]
    X, gm = _bern(case["n"])
    y = synthetic.bench_bernoulli_y(X)
    F = _offset(X)
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y, fixed_effects=F)
    assert abs(nll - case["nll"]) <= RTOL * abs(case["nll"]), (nll, case["nll"])
    np.testing.assert_allclose(g, case["grad"], rtol=RTOL)
    assert abs(gm.neg_log_likelihood(case["cov_pars"], y, fixed_effects=F) - case["nll"]) <= RTOL * abs(case["nll"])
    # without the offset the value differs (F enters the likelihood)
    assert abs(gm.neg_log_likelihood(case["cov_pars"], y) - case["nll"]) > 1.0
    gm.set_optim_params({"init_cov_pars": np.array(case["cov_pars"])})
    gf = gm.calc_gradient_f(fixed_effects=F)
    assert _close(gf, case["grad_f"]), np.max(np.abs(gf - case["grad_f"]))


def test_bernoulli_fit_with_offset_matches_reference(golden_lb):
    case = golden_lb["bernoulli_offset_fit"]
    X, gm = _bern(case["n"], cg=case["cg_delta_conv"])
    y = synthetic.bench_bernoulli_y(X)
    gm.fit(y, offset=_offset(X))
    np.testing.assert_allclose(gm.get_init_cov_pars(), case["init_cov_pars"], rtol=1e-12)
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-4)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-6 * abs(case["nll"])
    assert abs(gm.get_num_optim_iter() - case["num_it"]) <= 1
    # the boosting step after OptimCovPar(nullptr, score): the gradient wrt the score is finite
    gf = gm.calc_gradient_f(fixed_effects=_offset(X))
    assert np.all(np.isfinite(gf))


def test_gaussian_latent_with_offset_matches_reference(golden_lb):
    case = golden_lb["gauss_latent_offset"]
    n = case["n"]
    X = synthetic.bench_coords(n)
    F = _offset(X)
    y = synthetic.bench_gaussian_y(n) + F
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia_latent", num_neighbors=30,
                 vecchia_ordering="random", seed=0)
    gm.set_optim_params({"cg_delta_conv": case["cg_delta_conv"], "init_aux_pars": np.array([case["aux"]])})
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y, fixed_effects=F)
    assert abs(nll - case["nll"]) <= RTOL * abs(case["nll"])
    np.testing.assert_allclose(g, case["grad"], rtol=RTOL)
    gm.set_optim_params({"init_cov_pars": np.array(case["cov_pars"])})
    gf = gm.calc_gradient_f(fixed_effects=F)
    assert _close(gf, case["grad_f"])


@pytest.mark.parametrize("name", ["vecchia_grad_f", "dense_grad_f"])
def test_gaussian_gradient_wrt_f_matches_reference(golden_lb, name):
    case = golden_lb[name]
    n = case["n"]
    X = synthetic.bench_coords(n)
    r = _offset(X) - synthetic.bench_gaussian_y(n)
    kw = dict(gp_coords=X, cov_function="exponential", gp_approx=case["spec"]["gp_approx"], seed=0)
    if kw["gp_approx"] == "vecchia":
        kw.update(num_neighbors=30, vecchia_ordering="random")
    gm = GPModel(**kw)
    gm.set_optim_params({"init_cov_pars": np.array(case["cov_pars"])})
    gf = gm.calc_gradient_f(y=r)
    np.testing.assert_allclose(gf, case["grad_f"], rtol=1e-9, atol=1e-9 * np.max(np.abs(case["grad_f"])))
