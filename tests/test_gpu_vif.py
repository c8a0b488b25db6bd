"""GPU parity for the full-scale Vecchia approximation ("VIF", gp_approx = "full_scale_vecchia" / "vif",
Gaussian likelihood, cholesky) through the C ABI.

Reference: the ordering and inducing points of re_model_template.h:348-357 (shuffle, then
CreateREComponentsFITC_FSA with the same generator), the residual Vecchia factor of
CalcCovFactorGradientVecchia (Vecchia_utils.cpp:1388-1617), CalcCovFactorFITC_FSA (re_model_template.h:
8770-8880), CalcYAux (:8898-8935), log det (:2698-2714), CalcGradPars_FITC_FSA_GaussLikelihood_Cluster_i
(:1985-2232). Fixtures: tests/golden/golden_vif.json (the reference itself, make_golden_vif.py), to which
the dense numpy oracle (oracle/vif_oracle.py) is pinned at ~1e-14 by test_oracle_vif.py.

Tolerances: inducing points bit-exact; nll 1e-9, gradient 1e-7 relative (fp64 MFMA GEMMs, explicit
inverse factors and fixed-order sums vs Eigen's sparse / dense products: rounding only); fits with the
reference's iteration counts, estimates to 1e-6.
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPBoostError, GPModel, synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_vif.json")) as _f:
    GOLDEN = json.load(_f)
EVAL = [k for k in GOLDEN if k.startswith("vif_")]
FITS = [k for k in GOLDEN if k.startswith("fit_")]


def _data(n):
    X = synthetic.bench_coords(n)
    return X, synthetic.bench_spatial_gaussian_y(X)


def _model(case, X, gp_approx="full_scale_vecchia"):
    sp = case["spec"]
    return GPModel(gp_coords=X, cov_function=sp["cov_fct"], cov_fct_shape=float(sp["shape"]), gp_approx=gp_approx,
                   num_ind_points=int(sp["num_ind_points"]), num_neighbors=int(sp["num_neighbors"]),
                   vecchia_ordering=sp["ordering"], ind_points_selection=sp["ind_points_selection"],
                   seed=int(sp["seed"]))


@pytest.mark.parametrize("name", EVAL)
def test_vif_matches_reference(name):
    case = GOLDEN[name]
    X, y = _data(case["n"])
    gm = _model(case, X)
    Z = gm.inducing_points()
    ref_z = np.array(case["ind_points"]).reshape(case["m"], -1)
    assert np.array_equal(Z, ref_z), np.max(np.abs(Z - ref_z))
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= 1e-9 * abs(case["nll"]), (nll, case["nll"])
    np.testing.assert_allclose(g, case["grad"], rtol=1e-7, atol=1e-9 * abs(case["nll"]))
    nll_p, g_p, s2 = gm.neg_log_likelihood_and_grad(case["cov_pars"], y, profile_sigma2=True)
    assert abs(nll_p - case["nll_profiled"]) <= 1e-9 * abs(case["nll_profiled"])
    np.testing.assert_allclose(g_p, case["grad_profiled"], rtol=1e-7, atol=1e-9 * abs(case["nll_profiled"]))
    assert abs(s2 - case["sigma2_profiled"]) <= 1e-9 * abs(case["sigma2_profiled"])
    # the objective without the gradient is the same number
    assert gm.neg_log_likelihood(case["cov_pars"], y) == nll


def test_vif_alias_and_defaults():
    """gp_approx = "vif" is the same model (re_model_template.h:204-206); num_neighbors / num_ind_points
    default to 30 / 200 (:288-297, 320-330)."""
    case = GOLDEN["vif_exp_n2000_m50_nn10"]
    X, y = _data(case["n"])
    a = _model(case, X).neg_log_likelihood_and_grad(case["cov_pars"], y)
    b = _model(case, X, gp_approx="vif").neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert a[0] == b[0] and np.array_equal(a[1], b[1])
    gm = GPModel(gp_coords=X, gp_approx="vif", cov_function="exponential")
    assert gm.inducing_points().shape == (200, 2)


def test_vif_gradient_finite_differences():
    case = GOLDEN["vif_matern15_n2000_m100_nn20"]
    X, y = _data(case["n"])
    gm = _model(case, X)
    cp = np.array(case["cov_pars"])
    _, g, _ = gm.neg_log_likelihood_and_grad(cp, y)
    h = 1e-5
    for k in range(3):
        e = np.zeros(3)
        e[k] = h
        fd = (gm.neg_log_likelihood(cp * np.exp(e), y) - gm.neg_log_likelihood(cp * np.exp(-e), y)) / (2 * h)
        # original-scale log-parameters: d/dlog sigma1^2 of the transformed var = sigma1^2 / sigma^2, the
        # nugget enters both; compare the finite difference with the chain rule of the transformed gradient
        if k == 0:
            ref = g[0] - g[1]
        elif k == 1:
            ref = g[1]
        else:
            ref = -g[2]
        assert abs(fd - ref) <= 1e-4 * max(1.0, abs(ref)), (k, fd, ref)


@pytest.mark.parametrize("name", FITS)
def test_vif_fit_matches_reference(name):
    case = GOLDEN[name]
    X, y = _data(case["n"])
    gm = _model(case, X)
    gm.fit(y)
    np.testing.assert_allclose(gm.get_init_cov_pars(), case["init_cov_pars"], rtol=1e-12)
    assert gm.get_num_optim_iter() == case["num_it"]
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-6)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-9 * abs(case["nll"])


def test_vif_edge_cases_vs_oracle():
    """Tiny n (num_neighbors capped at n - 1, rows with fewer neighbours), one neighbour, m close to n,
    against the dense oracle."""
    from oracle import oracle as O
    from oracle.vif_oracle import vif_nll_grad
    for n, m, nn in [(30, 10, 40), (200, 20, 1), (120, 100, 12)]:
        X, y = _data(n)
        gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="full_scale_vecchia", num_ind_points=m,
                     num_neighbors=nn, seed=2)
        cp = [0.3, 1.1, 0.2]
        nll, g, _ = gm.neg_log_likelihood_and_grad(cp, y)
        perm, Z, _ = O.vif_inducing_points(X, m, "kmeans++", 2, True)
        xv = X[perm]
        nb = O.find_neighbors(xv, min(nn, n - 1))
        o = vif_nll_grad(xv, y[perm], nb, Z, 0, O.transform(0, cp), mode=0)
        assert abs(nll - o["nll"]) <= 1e-9 * abs(o["nll"]), (n, m, nn, nll, o["nll"])
        np.testing.assert_allclose(g, o["grad"], rtol=1e-7, atol=1e-9 * abs(o["nll"]))


def test_vif_refusals():
    X = synthetic.bench_coords(300)
    with pytest.raises(GPBoostError, match="iterative"):
        GPModel(gp_coords=X, gp_approx="full_scale_vecchia", num_ind_points=20, matrix_inversion_method="iterative")
    with pytest.raises(GPBoostError, match="random"):   # non-Gaussian VIF: kmeans++ / cover tree only (reference)
        GPModel(gp_coords=X, gp_approx="vif", num_ind_points=20, likelihood="bernoulli_logit",
                ind_points_selection="random")
    with pytest.raises(GPBoostError, match="num_neighbors"):
        GPModel(gp_coords=X, gp_approx="vif", num_ind_points=20, num_neighbors=60)
    gm = GPModel(gp_coords=X, gp_approx="vif", num_ind_points=20, num_neighbors=10)
    y = synthetic.bench_spatial_gaussian_y(X)
    gm.set_prediction_data(vecchia_pred_type="latent_order_obs_first_cond_obs_only")   # re_model_template.h:3761-3763
    with pytest.raises(GPBoostError, match="latent process"):
        gm.predict(y=y, gp_coords_pred=X[:5], cov_pars=[0.3, 1.0, 0.1])


@pytest.mark.parametrize("name", ["vif_matern15_n2000_m100_nn20", "vif_matern25_n3000_m200_nn30"])
def test_vif_row_forms_agree(monkeypatch, name):
    """The residual rows by the MFMA Gram form (neighbour sets <= 32, default) and by the LDS-staged VALU
    form (GPBOOST_AMD_VIF_ROWS=lds; used for nn > 31): the same factor up to summation order."""
    case = GOLDEN[name]
    X, y = _data(case["n"])
    out = {}
    for form in ("lds", "mfma"):
        monkeypatch.setenv("GPBOOST_AMD_VIF_ROWS", form)
        out[form] = _model(case, X).neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert abs(out["lds"][0] - out["mfma"][0]) <= 1e-11 * abs(out["lds"][0])
    np.testing.assert_allclose(out["mfma"][1], out["lds"][1], rtol=1e-9)


def test_vif_many_neighbours_vs_oracle():
    """nn = 40 > 31: the LDS-staged row form (neighbour sets beyond one 32-point MFMA tile pair)."""
    from oracle import oracle as O
    from oracle.vif_oracle import vif_nll_grad
    n, m, nn = 1500, 60, 40
    X, y = _data(n)
    gm = GPModel(gp_coords=X, cov_function="matern", cov_fct_shape=1.5, gp_approx="full_scale_vecchia",
                 num_ind_points=m, num_neighbors=nn, seed=4)
    cp = [0.2, 1.0, 0.15]
    nll, g, _ = gm.neg_log_likelihood_and_grad(cp, y)
    perm, Z, _ = O.vif_inducing_points(X, m, "kmeans++", 4, True)
    xv = X[perm]
    nb = O.find_neighbors(xv, nn)
    o = vif_nll_grad(xv, y[perm], nb, Z, 1, O.transform(1, cp), mode=0)
    assert abs(nll - o["nll"]) <= 1e-9 * abs(o["nll"]), (nll, o["nll"])
    np.testing.assert_allclose(g, o["grad"], rtol=1e-7, atol=1e-9 * abs(o["nll"]))
