"""GPU parity for the latent Vecchia path with matrix_inversion_method = "cholesky" (the reference's exact
Laplace-Vecchia branch, likelihoods.h:2935-2955, 3052-3070, 5207-5336, 6751-6811) through the C ABI: the sparse
Cholesky of Sigma^-1 + W (csrc/sparse_chol.{h,hip}, csrc/latent_chol.cpp).

Fixtures: tests/golden/golden_latent_chol.json (the reference itself, make_golden_latent_chol.py): nll + gradient
for five likelihoods and four covariance functions at n = 2000 and n = 20000, the R tests' values with
num_neighbors = n - 1 (probit 67.18342059, vecchia_latent 124.2549533, TOLERANCE_STRICT 1e-5 there), an L-BFGS
fit, the gradient wrt F and predictions. Both sides are exact sparse / dense algebra (no stochastic terms): nll
within 1e-9 relative, gradients 1e-7, fits with the reference's iteration count, predictions 1e-8. At
BASELINE.json's n = 100k (no reference value: the reference needs hours there) the gradient is checked against
central finite differences of the exact nll and repeat evaluations must be bitwise identical.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_latent_chol.json")) as _f:
    GOLDEN = json.load(_f)


def _data(kind, n):
    from gpboost_amd import synthetic
    if kind == "rtest_probit":
        return synthetic.rtest_bernoulli_probit_y(n)
    if kind == "rtest_gauss":
        return synthetic.rtest_gaussian_y(n)
    X = synthetic.bench_coords(n)
    if kind == "bench_gamma":
        return X, synthetic.bench_gamma_y(X)
    if kind == "bench_pois":
        return X, synthetic.bench_poisson_y(X)
    if kind == "bench_gauss":
        return X, synthetic.bench_gaussian_y(n)
    return X, synthetic.bench_bernoulli_y(X)


def _model(X, sp, aux=None, mim="cholesky"):
    from gpboost_amd import GPModel
    lik = sp["likelihood"]
    gm = GPModel(gp_coords=X, likelihood=lik, cov_function=sp["cov_fct"], cov_fct_shape=float(sp["shape"]),
                 gp_approx=sp["gp_approx"], num_neighbors=int(sp["num_neighbors"]), vecchia_ordering=sp["ordering"],
                 matrix_inversion_method=mim, seed=0)
    params = {}
    if aux is not None:
        params["init_aux_pars"] = [float(aux)]
        params["estimate_aux_pars"] = True
    if params:
        gm.set_optim_params(params)
    return gm


def _of(kind):
    return [k for k in GOLDEN if GOLDEN[k]["kind"] == kind]


@pytest.mark.parametrize("name", _of("eval"))
def test_latent_chol_nll_grad_match_reference(name):
    case = GOLDEN[name]
    X, y = _data(case["data"], case["n"])
    gm = _model(X, case["spec"], case["aux"])
    nll = gm.neg_log_likelihood(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= 1e-9 * abs(case["nll"]), (nll, case["nll"])
    nll2, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert abs(nll2 - case["nll"]) <= 1e-9 * abs(case["nll"])
    ref = np.asarray(case["grad"])
    assert g.shape == ref.shape, (g, ref)
    np.testing.assert_allclose(g, ref, rtol=1e-7, atol=1e-9 * abs(case["nll"]))
    if "r_expected_nll" in case:   # the R tests' own value (TOLERANCE_STRICT)
        assert abs(nll - case["r_expected_nll"]) < 1e-5


def test_latent_chol_fit_matches_reference():
    case = GOLDEN["fit_logit_m20_n500"]
    X, y = _data(case["data"], case["n"])
    gm = _model(X, case["spec"])
    gm.fit(y)
    np.testing.assert_allclose(gm.get_init_cov_pars(), case["init_cov_pars"], rtol=1e-12)
    assert gm.get_num_optim_iter() == case["num_it"]
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-6)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-9 * abs(case["nll"])


def test_latent_chol_gradient_wrt_fixed_effects():
    case = GOLDEN["gradf_pois_m20_n1000"]
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


@pytest.mark.parametrize("name", _of("pred"))
def test_latent_chol_predict_matches_reference(name):
    from gpboost_amd import synthetic
    case = GOLDEN[name]
    X, y = _data(case["data"], case["n"])
    npred = case["npred"]
    xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    if case["dup5"]:
        xp[:5] = X[:5]
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


def test_latent_chol_matches_dense_laplace_with_all_neighbours():
    """num_neighbors = n - 1 makes the Vecchia approximation exact: the Cholesky path then equals the dense Laplace
    path (gp_approx = "none") for every likelihood (n = 150, random ordering)."""
    from gpboost_amd import GPModel, synthetic
    n = 150
    X = synthetic.bench_coords(n)
    for lik, y in [("bernoulli_logit", synthetic.bench_bernoulli_y(X)), ("poisson", synthetic.bench_poisson_y(X))]:
        sp = dict(likelihood=lik, cov_fct="exponential", shape=0.5, gp_approx="vecchia", num_neighbors=n - 1,
                  ordering="random")
        a = _model(X, sp).neg_log_likelihood_and_grad([0.9, 0.15], y)
        b = GPModel(gp_coords=X, likelihood=lik, cov_function="exponential").neg_log_likelihood_and_grad([0.9, 0.15], y)
        assert abs(a[0] - b[0]) <= 1e-8 * abs(b[0]), (a[0], b[0])
        np.testing.assert_allclose(a[1], b[1], rtol=1e-6, atol=1e-8 * abs(b[0]))


def test_latent_chol_edge_cases():
    """Tiny n (one supernode, n <= m), one neighbour, and repeated evaluations with a warm mode: against the numpy
    oracle (dense restatement)."""
    from oracle import oracle as O
    from oracle.latent_chol_oracle import LatentCholOracle
    from gpboost_amd import synthetic
    for n, m, lik in [(5, 3, "bernoulli_logit"), (400, 1, "bernoulli_logit"), (50, 49, "gaussian"), (700, 8, "poisson")]:
        X = synthetic.bench_coords(n)
        y = {"gaussian": synthetic.bench_gaussian_y(n), "poisson": synthetic.bench_poisson_y(X)}.get(
            lik, synthetic.bench_bernoulli_y(X))
        mm = min(m, n - 1)
        sp = dict(likelihood=lik, cov_fct="exponential", shape=0.5, num_neighbors=m, ordering="random",
                  gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia")
        gm = _model(X, sp, 0.4 if lik == "gaussian" else None)
        nll, g, _ = gm.neg_log_likelihood_and_grad([0.9, 0.2], y)
        perm, xv, nb = O.vecchia_setup(X, mm, 0, True)
        ref = LatentCholOracle(xv, y[perm], nb, 0, O.transform_latent(0, [0.9, 0.2]), lik, aux=0.4)
        rg, _ = ref.grad()
        assert abs(nll - ref.nll) <= 1e-9 * abs(ref.nll), (n, m, lik, nll, ref.nll)
        np.testing.assert_allclose(g, rg, rtol=1e-7, atol=1e-9 * abs(ref.nll))


@pytest.mark.parametrize("lik", ["bernoulli_logit", "gaussian"])
def test_latent_chol_100k_fd_gradient_and_determinism(lik):
    """BASELINE.json n = 100k, m = 30 (config 5 for bernoulli_logit, the vecchia_latent form of config 3): the
    analytic gradient against central differences of the exact nll in log-parameters (step 1e-4; the O(h^2) error
    and the nll's rounding bound the agreement at ~1e-6 relative), bitwise-identical repeat evaluations."""
    from gpboost_amd import synthetic
    n = 100_000
    X = synthetic.bench_coords(n)
    y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
    sp = dict(likelihood=lik, cov_fct="exponential", shape=0.5, num_neighbors=30, ordering="random",
              gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia")
    aux = 0.1 if lik == "gaussian" else None
    gm = _model(X, sp, aux)
    cp = np.array([1.0, 0.1])
    a = gm.neg_log_likelihood_and_grad(cp, y)
    b = gm.neg_log_likelihood_and_grad(cp, None)
    assert a[0] == b[0] and np.array_equal(a[1], b[1])
    assert np.isfinite(a[0]) and np.all(np.isfinite(a[1]))
    h = 1e-4
    for k in range(2):
        e = np.zeros(2)
        e[k] = h
        fp = gm.neg_log_likelihood(cp * np.exp(e), None)
        fm = gm.neg_log_likelihood(cp * np.exp(-e), None)
        fd = (fp - fm) / (2 * h)
        ga = a[1][k] if k == 0 else -a[1][k]   # the gradient is wrt log(phi), phi = 1 / range (exponential)
        assert abs(fd - ga) <= 2e-6 * max(abs(ga), 1e-3 * abs(a[0])), (k, fd, ga)
