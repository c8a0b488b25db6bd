"""GPU parity of latent-model Vecchia predictions through the C ABI
(GPB_PredictREModel): vecchia_latent (gaussian) and bernoulli_logit under the iterative methods,
prediction type latent_order_obs_first_cond_obs_only (the reference default for latent models).

Reference fixtures: tests/golden/golden_latent_pred.json (make_golden_latent_pred.py: the reference's
own Predict, re_model_template.h:3146 -> PredictLaplaceApproxVecchia likelihoods.h:6576-6813).
* means = -Bpo mode: deterministic given the mode; at cg_delta_conv = 1e-10 the mode is converged and
  the means match at 1e-6 (the north-star tolerance); at the default 1e-2 both sides stop their PCG
  solves at the same iteration, so they agree to the rounding sensitivity of the Newton solves
  (bounded here at 1e-4 of the largest mean);
* variances: Dp plus a simulation term (nsim_var_pred draws; the reference's draws come from
  thread-seeded mt19937 streams, ours from a counter-based generator), so they are compared
  statistically: the fixture holds the reference at nsim = 20000, the GPU runs nsim = 4000, and the
  bound is 6 standard errors of the two sample variances, sqrt(2 / nsim) relative each, per point,
  plus a 1 % bound on the average relative difference over all prediction points.
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPModel, GPBoostError, synthetic

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(HERE, "golden", "golden_latent_pred.json")) as f:
        return json.load(f)


def _setup(case):
    n, nu = case["n"], case["nu"]
    X = synthetic.repeated_coords(n, nu) if nu else synthetic.bench_coords(n)
    lik = case["lik"]
    y = synthetic.bench_bernoulli_y(X) if lik == "bernoulli_logit" else synthetic.bench_gaussian_y(n)
    npred = case["npred"]
    Xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    sp = case["spec"]
    gm = GPModel(gp_coords=X, likelihood=lik, cov_function="exponential", gp_approx=sp["gp_approx"],
                 num_neighbors=int(sp["num_neighbors"]), vecchia_ordering="random",
                 matrix_inversion_method="iterative", seed=0)
    params = dict(num_rand_vec_trace=int(sp["num_rand_vec_trace"]), cg_delta_conv=float(sp.get("cg_delta_conv", 1e-2)))
    if "aux_pars" in sp:
        params["init_aux_pars"] = [float(sp["aux_pars"])]
    gm.set_optim_params(params)
    return gm, X, y, Xp


@pytest.mark.parametrize("name,tol", [("bern_n2000_tight", 1e-6), ("gauss_n2000_tight", 1e-6),
                                      ("bern_rep_n3000_tight", 1e-6), ("bern_n2000_default", 1e-4),
                                      ("bern_n100k_default", 1e-4)])
def test_latent_pred_mean_matches_reference(golden, name, tol):
    if name not in golden:
        pytest.skip("fixture not generated (make_golden_latent_pred.py --big)")
    case = golden[name]
    gm, X, y, Xp = _setup(case)
    pred = gm.predict(y=y, gp_coords_pred=Xp, cov_pars=case["cov_pars"], predict_response=False)
    ref = np.asarray(case["mean"])
    assert pred["var"] is None
    np.testing.assert_allclose(pred["mu"], ref, rtol=tol, atol=tol * np.abs(ref).max())


@pytest.mark.parametrize("name", ["bern_n2000_tight", "gauss_n2000_tight"])
def test_latent_pred_var_statistical(golden, name):
    case = golden[name]
    gm, X, y, Xp = _setup(case)
    nsim = 4000
    gm.set_prediction_data(nsim_var_pred=nsim)
    pred = gm.predict(y=y, gp_coords_pred=Xp, cov_pars=case["cov_pars"], predict_var=True, predict_response=False)
    ref_mu, ref_var = np.asarray(case["mean"]), np.asarray(case["var"])
    np.testing.assert_allclose(pred["mu"], ref_mu, rtol=1e-6, atol=1e-6 * np.abs(ref_mu).max())
    se = np.sqrt(2. / nsim + 2. / case["nsim"])   # relative standard error of the two sample variances
    rel = (pred["var"] - ref_var) / ref_var
    assert np.all(np.abs(rel) <= 6 * se), (np.abs(rel).max(), 6 * se)
    assert abs(rel.mean()) <= 0.01, rel.mean()
    assert np.all(pred["var"] > 0)


def test_latent_gaussian_response_adds_error_variance(golden):
    case = golden["gauss_n2000_tight"]
    gm, X, y, Xp = _setup(case)
    gm.set_prediction_data(nsim_var_pred=64)
    lat = gm.predict(y=y, gp_coords_pred=Xp[:50], cov_pars=case["cov_pars"], predict_var=True, predict_response=False)
    rsp = gm.predict(y=y, gp_coords_pred=Xp[:50], cov_pars=case["cov_pars"], predict_var=True, predict_response=True)
    np.testing.assert_array_equal(lat["mu"], rsp["mu"])
    # same draws are not reused across calls (fresh seed per call): compare through the statistical bound
    aux = float(case["spec"]["aux_pars"])
    rel = (rsp["var"] - aux - lat["var"]) / lat["var"]
    assert np.abs(rel).max() < 6 * np.sqrt(4. / 64)


def test_latent_bernoulli_response_probabilities(golden):
    # response means by the reference's adaptive Gauss-Hermite rule (30 nodes) over the simulated
    # latent variances; the variance's sampling error moves a probability by |dp/dvar| dvar <~ 5e-4
    # per standard error, so 3e-3 absolute is ~6 standard errors; var = p (1 - p) exactly
    case = golden["bern_n2000_tight_response"]
    gm, X, y, Xp = _setup(case)
    gm.set_prediction_data(nsim_var_pred=4000)
    pred = gm.predict(y=y, gp_coords_pred=Xp, cov_pars=case["cov_pars"], predict_var=True, predict_response=True)
    ref = np.asarray(case["mean"])
    assert np.all((pred["mu"] > 0) & (pred["mu"] < 1))
    np.testing.assert_allclose(pred["mu"], ref, rtol=0, atol=3e-3)
    assert abs((pred["mu"] - ref).mean()) < 5e-4
    np.testing.assert_allclose(pred["var"], pred["mu"] * (1 - pred["mu"]), rtol=1e-14, atol=0)


def test_latent_response_cov_mat_refused(golden):
    case = golden["bern_n2000_default"]
    gm, X, y, Xp = _setup(case)
    with pytest.raises(GPBoostError, match="covariance matrices"):
        gm.predict(y=y, gp_coords_pred=Xp[:10], cov_pars=case["cov_pars"], predict_cov_mat=True,
                   predict_response=True)


def _cov_bound(ref, nsim_ours, nsim_ref):
    # standard error of a sample covariance entry: sqrt((c_ii c_jj + c_ij^2) / nsim) (Gaussian draws),
    # with the reference's total covariance as a conservative stand-in for its simulated part
    d = np.diag(ref)
    return np.sqrt((np.outer(d, d) + ref ** 2) * (1. / nsim_ours + 1. / nsim_ref))


@pytest.mark.parametrize("name", ["bern_n2000_tight_cov", "bern_n2000_tight_condall_cov"])
def test_latent_pred_cov_statistical(golden, name):
    """Latent predictive covariance matrices (PredictLaplaceApproxVecchia, likelihoods.h:6651-6740:
    (1/nsim) sum (Bp^-1 Bpo z)(.)^T + Bp^-1 diag(Dp) Bp^-T), cond_obs_only and cond_all, against the
    reference at nsim = 20000: means at 1e-6, every entry within 6 standard errors of the two sample
    covariances, the matrix symmetric with a positive diagonal."""
    case = golden[name]
    gm, X, y, Xp = _setup(case)
    if "vecchia_pred_type" in case["spec"]:
        gm.set_prediction_data(vecchia_pred_type=case["spec"]["vecchia_pred_type"])
    nsim = 4000
    gm.set_prediction_data(nsim_var_pred=nsim)
    pred = gm.predict(y=y, gp_coords_pred=Xp, cov_pars=case["cov_pars"], predict_cov_mat=True, predict_response=False)
    ref_mu = np.asarray(case["mean"])
    np.testing.assert_allclose(pred["mu"], ref_mu, rtol=1e-6, atol=1e-6 * np.abs(ref_mu).max())
    npred = case["npred"]
    ref = np.asarray(case["cov"]).reshape(npred, npred)
    c = pred["cov"]
    np.testing.assert_allclose(c, c.T, rtol=0, atol=1e-12 * np.abs(c).max())
    assert np.all(np.diag(c) > 0)
    bound = 6 * _cov_bound(ref, nsim, case["nsim"])
    assert np.all(np.abs(c - ref) <= bound), np.max(np.abs(c - ref) / bound)


@pytest.mark.parametrize("name", ["bern_n2000_tight_condall", "gauss_n2000_tight_condall"])
def test_latent_pred_cond_all(golden, name):
    """latent_order_obs_first_cond_all for latent models: mean = -Bp^-1 Bpo mode (likelihoods.h:6613-6616)
    at 1e-6; variances statistically as in test_latent_pred_var_statistical."""
    case = golden[name]
    gm, X, y, Xp = _setup(case)
    nsim = 4000
    gm.set_prediction_data(vecchia_pred_type="latent_order_obs_first_cond_all", nsim_var_pred=nsim)
    pred = gm.predict(y=y, gp_coords_pred=Xp, cov_pars=case["cov_pars"], predict_var=True, predict_response=False)
    ref_mu, ref_var = np.asarray(case["mean"]), np.asarray(case["var"])
    np.testing.assert_allclose(pred["mu"], ref_mu, rtol=1e-6, atol=1e-6 * np.abs(ref_mu).max())
    se = np.sqrt(2. / nsim + 2. / case["nsim"])
    rel = (pred["var"] - ref_var) / ref_var
    assert np.all(np.abs(rel) <= 6 * se), (np.abs(rel).max(), 6 * se)
    assert abs(rel.mean()) <= 0.01, rel.mean()
