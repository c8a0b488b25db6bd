"""GPU parity for the GPBoost algorithm's covariance update: three consecutive
boosting rounds of REModel::OptimCovPar(..., called_in_GPBoost_algorithm=true,
reuse_learning_rates_gp_model) + REModel::CalcGradient(..., calc_cov_factor=false) on the scores
F_r = scale_r * F, as the boosting objective runs them (regression_objective.hpp:153-182), through
GPB_OptimCovParBoosting / GPB_CalcGradientF. Fixtures: tests/golden/golden_boost.json
(make_golden_boost.py, the reference itself).

What it pins: the L-BFGS memory carried from one round into the next (reuse = 1: the first direction
of round r + 1 is -H g at step 1, re_model_template.h:880-881, LBFGS.h:158-171) against a fresh
solver every round (reuse = 0), the offset not being saved in boosting mode, and for the Laplace
model the mode carried across objective evaluations and rounds (likelihoods.h:2782-2789).
Tolerances: exact Gaussian paths 1e-6 on the estimates (north-star tolerance; the iteration counts
must match exactly), the gradient wrt F 1e-6 of its largest entry; bernoulli_logit at cg_delta_conv =
1e-8 with the reference's probe streams: 1e-6.
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPModel, synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(HERE, "golden", "golden_boost.json")) as f:
        return json.load(f)


def _score(X):
    return 0.5 * np.sin(3 * X[:, 0]) - 0.3 * X[:, 1]


def _close(a, b, rtol=1e-6):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.max(np.abs(a - b)) <= rtol * max(np.max(np.abs(b)), 1.0)


@pytest.mark.parametrize("name", ["gauss_vecchia_reuse1", "gauss_vecchia_reuse0", "gauss_dense_reuse1",
                                  "gauss_dense_reuse0"])
def test_gaussian_boosting_rounds_match_reference(golden, name):
    case = golden[name]
    n = case["n"]
    X = synthetic.bench_coords(n)
    y = synthetic.bench_gaussian_y(n)
    kw = dict(gp_coords=X, cov_function="exponential", gp_approx=case["spec"]["gp_approx"], seed=0)
    if kw["gp_approx"] == "vecchia":
        kw.update(num_neighbors=30, vecchia_ordering="random")
    gm = GPModel(**kw)
    for scale, ref in zip(golden["scales"], case["rounds"]):
        g = scale * _score(X) - y           # the boosting gradient F - label (regression_objective.hpp:159-162)
        gm.optim_cov_par_boosting(y=g, reuse_learning_rates=bool(case["reuse"]))
        assert gm.get_num_optim_iter() == ref["num_it"], (scale, gm.get_num_optim_iter(), ref["num_it"])
        np.testing.assert_allclose(gm.get_cov_pars(), ref["cov_pars"], rtol=1e-6)
        gf = gm.calc_gradient_f(y=g, calc_cov_factor=False)
        assert _close(gf, ref["grad_f"]), np.max(np.abs(gf - ref["grad_f"]))
    # boosting mode does not save the score as the model's offset (re_model_template.h:1051)
    import ctypes
    from gpboost_amd.basic import lib, _dp
    buf = np.zeros(n)
    assert lib().GPB_GetOffsetData(gm.handle, _dp(buf)) == -1


def test_reuse_changes_the_trajectory(golden):
    """The two fixtures differ from round 2 on: the carried L-BFGS memory is what the reuse pins."""
    a = golden["gauss_vecchia_reuse1"]["rounds"]
    b = golden["gauss_vecchia_reuse0"]["rounds"]
    assert a[0]["num_it"] == b[0]["num_it"]
    assert a[1]["num_it"] != b[1]["num_it"]


def test_bernoulli_boosting_rounds_match_reference(golden):
    case = golden["bernoulli_cg1e-8"]
    n = case["n"]
    X = synthetic.bench_coords(n)
    yb = synthetic.bench_bernoulli_y(X)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", likelihood="bernoulli_logit",
                 num_neighbors=30, vecchia_ordering="random", seed=0)
    gm.set_optim_params({"cg_delta_conv": case["cg_delta_conv"]})
    for r, (scale, ref) in enumerate(zip(golden["scales"], case["rounds"])):
        F = scale * _score(X)
        gm.optim_cov_par_boosting(y=yb if r == 0 else None, fixed_effects=F, reuse_learning_rates=True)
        assert gm.get_num_optim_iter() == ref["num_it"], (scale, gm.get_num_optim_iter(), ref["num_it"])
        np.testing.assert_allclose(gm.get_cov_pars(), ref["cov_pars"], rtol=1e-6)
        assert abs(gm.get_current_neg_log_likelihood() - ref["nll"]) <= 1e-6 * abs(ref["nll"])
        gf = gm.calc_gradient_f(fixed_effects=F, calc_cov_factor=False)
        assert _close(gf, ref["grad_f"]), np.max(np.abs(gf - ref["grad_f"]))


# ---- regression tests of the prediction / evaluation fixes of this round

def test_latent_response_prediction_applies_offset_before_the_link():
    """fixed_effects_pred joins the latent mean before the response transform
    (re_model_template.h:3929-3946): bernoulli probabilities stay in [0, 1] and move with F_pred."""
    n = 1000
    X = synthetic.bench_coords(n)
    yb = synthetic.bench_bernoulli_y(X)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", likelihood="bernoulli_logit",
                 num_neighbors=30, vecchia_ordering="random", seed=0)
    gm.neg_log_likelihood([1.0, 0.1], yb)
    xp = synthetic.bench_coords(40)[:, ::-1] * 0.9 + 0.05
    base = gm.predict(gp_coords_pred=xp, cov_pars=[1.0, 0.1], predict_response=True, predict_var=True)["mu"]
    hi = gm.predict(gp_coords_pred=xp, cov_pars=[1.0, 0.1], predict_response=True, predict_var=True,
                    offset_pred=np.full(40, 20.0))
    lo = gm.predict(gp_coords_pred=xp, cov_pars=[1.0, 0.1], predict_response=True, predict_var=True,
                    offset_pred=np.full(40, -20.0))
    for r in (hi["mu"], lo["mu"], base):
        assert np.all((r >= 0.0) & (r <= 1.0))
    assert np.all(hi["mu"] > 0.999) and np.all(lo["mu"] < 0.001)
    np.testing.assert_allclose(hi["var"], hi["mu"] * (1.0 - hi["mu"]), rtol=1e-12, atol=1e-15)


def test_gaussian_latent_response_mean_is_shifted_by_the_offset():
    n = 800
    X = synthetic.bench_coords(n)
    y = synthetic.bench_gaussian_y(n)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia_latent", num_neighbors=30,
                 vecchia_ordering="random", seed=0)
    gm.set_optim_params({"init_aux_pars": np.array([0.1]), "cg_delta_conv": 1e-10})
    gm.neg_log_likelihood([1.0, 0.1], y)
    xp = synthetic.bench_coords(30)[:, ::-1] * 0.9 + 0.05
    F = np.linspace(-1.0, 1.0, 30)
    a = gm.predict(gp_coords_pred=xp, cov_pars=[1.0, 0.1], predict_response=True)["mu"]
    b = gm.predict(gp_coords_pred=xp, cov_pars=[1.0, 0.1], predict_response=True, offset_pred=F)["mu"]
    np.testing.assert_allclose(b, a + F, rtol=0, atol=1e-12)


def test_latent_prediction_uses_the_offset_saved_by_the_fit():
    """No offset at prediction time: the one saved by fit(offset=...) (re_model_template.h:3306-3312,
    4032-4039), i.e. the same predictions as passing it explicitly."""
    n = 800
    X = synthetic.bench_coords(n)
    yb = synthetic.bench_bernoulli_y(X)
    F = _score(X)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", likelihood="bernoulli_logit",
                 num_neighbors=30, vecchia_ordering="random", seed=0)
    gm.set_optim_params({"cg_delta_conv": 1e-8, "maxit": 3})
    gm.fit(yb, offset=F)
    xp = synthetic.bench_coords(25)[:, ::-1] * 0.9 + 0.05
    saved = gm.predict(gp_coords_pred=xp, predict_response=False)["mu"]
    given = gm.predict(gp_coords_pred=xp, predict_response=False, offset=F)["mu"]
    none = gm.predict(gp_coords_pred=xp, predict_response=False, offset=np.zeros(n))["mu"]
    np.testing.assert_allclose(saved, given, rtol=0, atol=1e-12)
    assert np.max(np.abs(saved - none)) > 1e-3
    # training-data random effects: the saved offset as well (GPB_PredictREModelTrainingDataRandomEffects)
    import ctypes
    from gpboost_amd.basic import lib, _dp
    cp = np.ascontiguousarray(gm.get_cov_pars())
    a, b = np.zeros(n), np.zeros(n)
    assert lib().GPB_PredictREModelTrainingDataRandomEffects(gm.handle, _dp(cp), None, _dp(a), None, False) == 0
    assert lib().GPB_PredictREModelTrainingDataRandomEffects(gm.handle, _dp(cp), None, _dp(b),
                                                             _dp(np.ascontiguousarray(F)), False) == 0
    np.testing.assert_allclose(a, b, rtol=0, atol=1e-12)


def test_eval_without_cov_pars_uses_the_initial_values():
    """GPB_EvalNegLogLikelihood(cov_pars = NULL) evaluates at the current (initialised) parameters
    (re_model.cpp:598-605)."""
    import ctypes
    from gpboost_amd.basic import lib, _dp
    n = 1500
    X = synthetic.bench_coords(n)
    y = synthetic.bench_gaussian_y(n)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=30,
                 vecchia_ordering="random", seed=0)
    v = ctypes.c_double(0)
    assert lib().GPB_EvalNegLogLikelihood(gm.handle, _dp(np.ascontiguousarray(y)), None, None, ctypes.byref(v)) == 0
    init = gm.get_init_cov_pars()
    assert np.all(init > 0)
    np.testing.assert_allclose(v.value, gm.neg_log_likelihood(init, y), rtol=1e-12)
