"""GPU parity for the Laplace likelihoods bernoulli_probit and poisson on both latent paths, through the
C ABI: Vecchia + iterative methods (PCG / SLQ / VADU, the same probe streams as the reference) and FITC
(cholesky). Reference: the likelihood's log-density and its first three derivatives (likelihoods.h
bernoulli_probit :8708, 9208, 9871, 10171; poisson :8730, 9230, 9904, 10200 with the normalizing constant
-sum log y!), response predictions (PredictResponse :7526-7569).

Fixtures: tests/golden/golden_latent_lik.json (the reference itself, make_golden_latent_lik.py), whose
R-test data cases are in turn pinned to the R tests' hard-coded nll values (test_oracle_fitc_laplace.py).
Tolerances as for bernoulli_logit: Vecchia nll / gradient 1e-6 relative (north star); FITC nll 1e-8,
gradient 1e-6, predictions 1e-7, fits to 1e-6 with the reference's iteration count.
"""
import json
import os

import numpy as np
import pytest

from conftest import lik_case_data

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_latent_lik.json")) as _f:
    GOLDEN = json.load(_f)


def _of(kind):
    return [k for k in GOLDEN if GOLDEN[k]["kind"] == kind]


def _vecchia(X, case):
    from gpboost_amd import GPModel
    gm = GPModel(gp_coords=X, likelihood=case["likelihood"], cov_function=case["cov_fct"],
                 cov_fct_shape=case["shape"], gp_approx="vecchia", num_neighbors=case["num_neighbors"],
                 vecchia_ordering=case["ordering"], matrix_inversion_method="iterative", seed=0)
    gm.set_optim_params(dict(num_rand_vec_trace=case["num_rand_vec_trace"],
                             seed_rand_vec_trace=case["seed_rand_vec_trace"], cg_delta_conv=case["cg_delta_conv"]))
    return gm


def _fitc(X, case):
    from gpboost_amd import GPModel
    sp = case["spec"]
    return GPModel(gp_coords=X, cov_function=sp["cov_fct"], cov_fct_shape=float(sp["shape"]), gp_approx="fitc",
                   num_ind_points=int(sp["num_ind_points"]), likelihood=case["likelihood"],
                   ind_points_selection=sp["ind_points_selection"], seed=int(sp["seed"]))


@pytest.mark.parametrize("name", _of("vecchia"))
def test_vecchia_iterative_matches_reference(name):
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    gm = _vecchia(X, case)
    nll = gm.neg_log_likelihood(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= 1e-6 * abs(case["nll"]), (nll, case["nll"])
    nll2, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], None)
    assert abs(nll2 - case["nll"]) <= 1e-6 * abs(case["nll"])
    ref = np.asarray(case["grad"])
    np.testing.assert_allclose(g, ref, rtol=1e-6, atol=1e-6 * np.abs(ref).max())


@pytest.mark.parametrize("name", _of("fitc"))
def test_fitc_matches_reference(name):
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    gm = _fitc(X, case)
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= 1e-8 * abs(case["nll"]), (nll, case["nll"])
    np.testing.assert_allclose(g, case["grad"], rtol=1e-6, atol=1e-8 * abs(case["nll"]))


@pytest.mark.parametrize("name", _of("fitc_fit"))
def test_fitc_fit_matches_reference(name):
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    gm = _fitc(X, case)
    gm.fit(y)
    np.testing.assert_allclose(gm.get_init_cov_pars(), case["init_cov_pars"], rtol=1e-12)
    assert gm.get_num_optim_iter() == case["num_it"]
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-6)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-8 * abs(case["nll"])


@pytest.mark.parametrize("name", _of("fitc_gradf"))
def test_fitc_gradient_wrt_fixed_effects(name):
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    fe = 0.3 * np.sin(3.0 * X[:, 0]) - 0.2
    gm = _fitc(X, case)
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y, fixed_effects=fe)
    assert abs(nll - case["nll"]) <= 1e-8 * abs(case["nll"])
    np.testing.assert_allclose(g, case["grad"], rtol=1e-6)
    gm.set_optim_params({"init_cov_pars": np.array(case["cov_pars"])})
    gf = gm.calc_gradient_f(fixed_effects=fe)
    ref = np.asarray(case["grad_f"])
    assert np.max(np.abs(gf - ref)) <= 1e-7 * max(1.0, np.max(np.abs(ref))), np.max(np.abs(gf - ref))


@pytest.mark.parametrize("name", _of("fitc_pred"))
def test_fitc_predict_matches_reference(name):
    from gpboost_amd import synthetic
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    npred = case["npred"]
    xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    gm = _fitc(X, case)
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


def test_vecchia_response_prediction_closed_form():
    """Vecchia latent predictions with predict_response: probit Phi(mu / sqrt(1 + var)) with variance
    p (1 - p), poisson exp(mu + var / 2) with variance pm ((e^var - 1) pm + 1) (likelihoods.h:7531-7569).
    The latent variance is a simulation estimate drawn anew by each predict call (nsim_var_pred), the
    latent mean is not: the transform is inverted on the response output and the recovered mean must equal
    the latent mean (poisson, exact) and the recovered variance the other call's estimate within its
    simulation noise."""
    from scipy.stats import norm
    from gpboost_amd import synthetic
    for name in ("vp_probit_m30_exp_tight", "vp_pois_m30_exp_tight"):
        case = GOLDEN[name]
        X, y = lik_case_data(case)
        gm = _vecchia(X, case)
        xp = synthetic.lcg_unif(80, 0.713).reshape(2, 40).T.copy()
        lat = gm.predict(y=y, gp_coords_pred=xp, cov_pars=case["cov_pars"], predict_var=True, predict_response=False)
        resp = gm.predict(y=y, gp_coords_pred=xp, cov_pars=case["cov_pars"], predict_var=True, predict_response=True)
        mu, var = np.asarray(lat["mu"]), np.asarray(lat["var"])
        pm, pv = np.asarray(resp["mu"]), np.asarray(resp["var"])
        if case["likelihood"] == "bernoulli_probit":
            np.testing.assert_allclose(pv, pm * (1. - pm), rtol=1e-14)
            z = norm.ppf(pm)
            ok = np.abs(z) > 0.2                                   # var recoverable away from p = 1/2
            v_rec = (mu[ok] / z[ok]) ** 2 - 1.
            np.testing.assert_allclose(v_rec, var[ok], rtol=0.1, atol=0.02)
        else:
            v_rec = np.log1p((pv / pm - 1.) / pm)
            np.testing.assert_allclose(np.log(pm) - 0.5 * v_rec, mu, rtol=1e-9, atol=1e-9)
            np.testing.assert_allclose(v_rec, var, rtol=0.1, atol=0.02)


def test_likelihood_response_checks():
    from gpboost_amd import GPBoostError, GPModel, synthetic
    X = synthetic.bench_coords(300)
    for lik, bad, msg in [("bernoulli_probit", np.full(300, 0.5), "0 or 1"), ("poisson", -np.ones(300), "y >= 0"),
                          ("poisson", np.full(300, 1.5), "integer")]:
        for approx in ("vecchia", "fitc"):
            kw = dict(num_neighbors=10, matrix_inversion_method="iterative") if approx == "vecchia" else dict(num_ind_points=20)
            gm = GPModel(gp_coords=X, likelihood=lik, gp_approx=approx, **kw)
            with pytest.raises(GPBoostError, match=msg):
                gm.neg_log_likelihood([1.0, 0.1], bad)


@pytest.mark.parametrize("name", ["fp_pois_gauss_n2500_m60_random", "fp_probit_matern15_n3000_m80"])
def test_fitc_gradient_g_forms_agree(monkeypatch, name):
    """G = M^-1 K_mn by the explicit inverse (default) or through the inverse Cholesky factor
    (GPBOOST_AMD_FITC_G=tri): the same nll bit for bit (G enters only the gradient) and gradients within
    1e-8 relative, on the worst-conditioned fixture (Gaussian kernel, Poisson information)."""
    case = GOLDEN[name]
    X, y = lik_case_data(case)
    out = {}
    for form in ("inv", "tri"):
        monkeypatch.setenv("GPBOOST_AMD_FITC_G", form)
        out[form] = _fitc(X, case).neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert out["inv"][0] == out["tri"][0]
    np.testing.assert_allclose(out["tri"][1], out["inv"][1], rtol=1e-8)
