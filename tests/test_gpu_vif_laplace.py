"""GPU parity for the full-scale Vecchia approximation ("VIF", gp_approx = "full_scale_vecchia") with a non-Gaussian
likelihood and matrix_inversion_method = "cholesky" (the reference's FSVA Laplace approximation: FindModePostRandEffCalcMLLFSVA
likelihoods.h:2316-2742, CalcGradNegMargLikelihoodLaplaceApproxFSVA :3886-4925) through the C ABI: VifLaplace
(csrc/vif_laplace.{h,hip}) on the VIF residual factor and the GPU sparse Cholesky.

Fixtures: tests/golden/golden_vif_laplace.json (the reference itself, make_golden_vif_laplace.py): nll + gradient for
bernoulli_logit / bernoulli_probit / poisson / gamma (with the shape gradient) over four covariance functions, m = 20-200
inducing points, 8-30 neighbours, n = 1000-20000; L-BFGS fits; latent / response predictions; the gradient wrt F (with fixed effects the reference's
covariance gradient evaluates its location-dependent terms at mode + F in data order, re_model_template.h:1859,
reproduced by VifLaplace::SetGradOffset). Both sides are exact algebra: nll
within 1e-9 relative (2e-9 for the smooth-kernel cases, whose residual factor the reference forms by cancellation,
cond(M) ~1e5-1e6), gradients 1e-7 (4e-7 there), fits with the reference's iteration counts. The dense restatement
(oracle/vif_laplace_oracle.py, pinned to the same fixtures by tests/test_oracle_vif_laplace.py) checks further cases.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_vif_laplace.json")) as _f:
    GOLDEN = json.load(_f)


def _data(kind, n):
    from gpboost_amd import synthetic
    X = synthetic.bench_coords(n)
    if kind == "bench_gamma":
        return X, synthetic.bench_gamma_y(X)
    if kind == "bench_pois":
        return X, synthetic.bench_poisson_y(X)
    return X, synthetic.bench_bernoulli_y(X)


def _model(X, sp, aux=None, mim="cholesky"):
    from gpboost_amd import GPModel
    gm = GPModel(gp_coords=X, likelihood=sp["likelihood"], cov_function=sp["cov_fct"], cov_fct_shape=float(sp["shape"]),
                 gp_approx="full_scale_vecchia", num_ind_points=int(sp["num_ind_points"]),
                 num_neighbors=int(sp["num_neighbors"]), ind_points_selection=sp["ind_points_selection"],
                 seed=int(sp["seed"]), matrix_inversion_method=mim)
    if aux is not None:
        gm.set_optim_params({"init_aux_pars": [float(aux)], "estimate_aux_pars": True})
    return gm


def _of(kind):
    return [k for k in GOLDEN if GOLDEN[k]["kind"] == kind]


def _tol(case):
    sp = case["spec"]
    smooth = sp["cov_fct"] == "gaussian" or (sp["cov_fct"] == "matern" and float(sp["shape"]) > 0.5)
    return (2e-9, 4e-7) if smooth else (1e-9, 1e-7)


@pytest.mark.parametrize("name", _of("eval"))
def test_vif_laplace_nll_grad_match_reference(name):
    case = GOLDEN[name]
    X, y = _data(case["data"], case["n"])
    gm = _model(X, case["spec"], case["aux"])
    tn, tg = _tol(case)
    nll = gm.neg_log_likelihood(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= tn * abs(case["nll"]), (nll, case["nll"])
    nll2, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert abs(nll2 - case["nll"]) <= tn * abs(case["nll"])
    ref = np.asarray(case["grad"])
    assert g.shape == ref.shape, (g, ref)
    np.testing.assert_allclose(g, ref, rtol=tg, atol=tg * np.abs(ref).max())
    if "ind_points" in case:
        np.testing.assert_array_equal(gm.inducing_points().ravel(), case["ind_points"])


@pytest.mark.parametrize("name", _of("fit"))
def test_vif_laplace_fit_matches_reference(name):
    case = GOLDEN[name]
    X, y = _data(case["data"], case["n"])
    gm = _model(X, case["spec"])
    gm.fit(y)
    np.testing.assert_allclose(gm.get_init_cov_pars(), case["init_cov_pars"], rtol=1e-12)
    assert gm.get_num_optim_iter() == case["num_it"]
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-6)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-9 * abs(case["nll"])


def test_vif_laplace_gradient_wrt_fixed_effects():
    case = GOLDEN["gradf_pois_m30_nn10_n1000"]
    X, y = _data(case["data"], case["n"])
    fe = 0.3 * np.sin(3.0 * X[:, 0]) - 0.2
    gm = _model(X, case["spec"])
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y, fixed_effects=fe)
    assert abs(nll - case["nll"]) <= 1e-9 * abs(case["nll"])
    np.testing.assert_allclose(g, case["grad"], rtol=1e-7)
    gm.set_optim_params({"init_cov_pars": np.array(case["cov_pars"])})
    gf = gm.calc_gradient_f(fixed_effects=fe)
    ref = np.asarray(case["grad_f"])
    assert np.max(np.abs(gf - ref)) <= 1e-8 * max(1.0, np.max(np.abs(ref))), np.max(np.abs(gf - ref))


@pytest.mark.parametrize("lik,cov,shape,m,nn,cp", [
    ("bernoulli_logit", "exponential", 0.5, 25, 12, (0.7, 0.2)),
    ("poisson", "matern", 2.5, 40, 20, (1.2, 0.08)),
    ("bernoulli_probit", "matern", 1.5, 10, 35, (0.5, 0.3)),
])
def test_vif_laplace_matches_oracle(lik, cov, shape, m, nn, cp):
    """The dense restatement at n = 600, the residual rows on both row-kernel forms (nn <= 31: the MFMA form,
    nn = 35: the LDS-staged form)."""
    from gpboost_amd import synthetic
    from oracle import oracle as O
    from oracle.vif_laplace_oracle import VifLaplaceOracle
    n = 600
    X = synthetic.bench_coords(n)
    y = synthetic.bench_poisson_y(X) if lik == "poisson" else synthetic.bench_bernoulli_y(X)
    sp = dict(likelihood=lik, cov_fct=cov, shape=shape, num_ind_points=m, num_neighbors=nn,
              ind_points_selection="kmeans++", seed=1)
    gm = _model(X, sp)
    nll, g, _ = gm.neg_log_likelihood_and_grad(list(cp), y)
    perm, Z, _ = O.vif_inducing_points(X, m, "kmeans++", 1, True)
    xv = X[perm]
    nb = O.find_neighbors(xv, nn)
    ct = O.cov_code(cov, shape)
    tr = O.transform_latent(ct, cp)
    o = VifLaplaceOracle(xv, y[perm], nb, Z, ct, tr[0], tr[1], lik)
    og, _ = o.grad()
    assert abs(nll - o.nll) <= 1e-9 * abs(o.nll), (nll, o.nll)
    np.testing.assert_allclose(g, og, rtol=1e-6, atol=1e-7 * np.abs(og).max())


def test_vif_laplace_refusals():
    from gpboost_amd import GPModel, synthetic
    from gpboost_amd.basic import GPBoostError
    X = synthetic.bench_coords(300)
    with pytest.raises(GPBoostError, match="random"):
        GPModel(gp_coords=X, likelihood="bernoulli_logit", gp_approx="full_scale_vecchia", num_ind_points=20,
                ind_points_selection="random")
    with pytest.raises(GPBoostError, match="iterative"):
        GPModel(gp_coords=X, likelihood="bernoulli_logit", gp_approx="full_scale_vecchia", num_ind_points=20,
                matrix_inversion_method="iterative")


def test_vif_laplace_default_method_is_cholesky_and_deterministic():
    from gpboost_amd import GPModel, synthetic
    X = synthetic.bench_coords(800)
    y = synthetic.bench_bernoulli_y(X)
    a = GPModel(gp_coords=X, likelihood="bernoulli_logit", gp_approx="full_scale_vecchia", num_ind_points=30,
                num_neighbors=10)
    b = GPModel(gp_coords=X, likelihood="bernoulli_logit", gp_approx="full_scale_vecchia", num_ind_points=30,
                num_neighbors=10, matrix_inversion_method="cholesky")
    ra = a.neg_log_likelihood_and_grad([1.0, 0.1], y)
    rb = b.neg_log_likelihood_and_grad([1.0, 0.1], y)
    rc = b.neg_log_likelihood_and_grad([1.0, 0.1], y)
    assert ra[0] == rb[0] == rc[0]
    np.testing.assert_array_equal(ra[1], rb[1])
    np.testing.assert_array_equal(rb[1], rc[1])


@pytest.mark.parametrize("name", _of("pred"))
def test_vif_laplace_predict_matches_reference(name):
    """PredictLaplaceApproxFSVA, Cholesky branch (likelihoods.h:6060-6130, 6478-6548): latent means, variances,
    covariance matrices (cond_obs_only / cond_all) and response probabilities at 1e-8."""
    from gpboost_amd import synthetic
    case = GOLDEN[name]
    X, y = _data(case["data"], case["n"])
    npred = case["npred"]
    xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    gm = _model(X, case["spec"])
    gm.set_prediction_data(vecchia_pred_type=case["vecchia_pred_type"])
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
