"""GPU parity for GPB_OptimCovPar (covariance-parameter estimation with "lbfgs").

Reference: REModel::OptimCovPar (re_model.cpp:339-401) -> OptimLinRegrCoefCovPar
(re_model_template.h:846-1700) -> OptimExternal / LBFGSpp (optim_utils.h:561-706). Fixtures:
tests/golden/golden_fit.json (make_golden_fit.py: the reference itself, Python-package default
settings) and the R-test golden of test_GPModel_gaussian_process.R:233-237.

The optimizer follows the reference's trajectory step for step (same initial values, line
search, inverse-Hessian updates, stopping rule), and the device objective matches the
reference's to ~1e-12 relative, so the exact paths must reproduce the iteration count and the
estimates to 1e-6 relative. Latent cases (Laplace + PCG / SLQ at cg_delta_conv = 1e-6): the
objective agrees to ~1e-7, so estimates are checked at 1e-4 relative.
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPModel, GPBoostError, synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden_fit():
    with open(os.path.join(HERE, "golden", "golden_fit.json")) as f:
        return json.load(f)


def _data(case):
    if case["data"] == "rtest_gaussian":
        return synthetic.rtest_gaussian_y(100)
    X = synthetic.bench_coords(case["n"])
    if case["data"] == "bench":
        return X, synthetic.bench_gaussian_y(case["n"])
    if case["spec"].get("likelihood") == "bernoulli_logit":
        return X, synthetic.bench_bernoulli_y(X)
    return X, synthetic.bench_gaussian_y(case["n"])


def _model(case, X):
    sp = case["spec"]
    kw = dict(gp_coords=X, cov_function=sp["cov_fct"], cov_fct_shape=float(sp.get("shape", 0.5)),
              gp_approx=sp["gp_approx"], likelihood=sp.get("likelihood", "gaussian"), seed=0)
    if sp["gp_approx"] != "none":
        kw.update(num_neighbors=sp["num_neighbors"], vecchia_ordering=sp["ordering"])
    if "matrix_inversion_method" in sp:
        kw["matrix_inversion_method"] = sp["matrix_inversion_method"]
    return GPModel(**kw)


def _params(case):
    sp = case["spec"]
    p = {}
    if "init_cov_pars" in sp:
        p["init_cov_pars"] = np.array([float(v) for v in sp["init_cov_pars"].split(",")])
    if "cg_delta_conv" in sp:
        p.update(cg_delta_conv=float(sp["cg_delta_conv"]), num_rand_vec_trace=int(sp["num_rand_vec_trace"]),
                 seed_rand_vec_trace=int(sp["seed_rand_vec_trace"]))
    return p


EXACT = ["rtest_dense_exponential", "rtest_vecchia_m30_random", "rtest_dense_matern15_init",
         "synth2000_vecchia_m30_exp", "synth2000_vecchia_m20_gaussian", "synth2000_vecchia_m30_matern25_init",
         "synth2000_dense_exp"]


@pytest.mark.parametrize("name", EXACT)
def test_fit_matches_reference_exact(golden_fit, name):
    case = golden_fit[name]
    X, Y = _data(case)
    gm = _model(case, X)
    gm.fit(Y, params=_params(case))
    est = gm.get_cov_pars()
    assert gm.get_num_optim_iter() == case["num_it"]
    np.testing.assert_allclose(est, case["cov_pars"], rtol=1e-6)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-9 * abs(case["nll"])


def test_fit_r_golden():
    # test_GPModel_gaussian_process.R:233-237 (lbfgs, default settings)
    X, Y = synthetic.rtest_gaussian_y(100)
    gm = GPModel(gp_coords=X, cov_function="exponential")
    gm.fit(Y)
    est = gm.get_cov_pars()
    assert np.sum(np.abs(est - np.array([0.03784221, 1.07390943, 0.11451432]))) < 1e-2
    assert abs(gm.get_current_neg_log_likelihood() - 122.7771373) < 1e-2
    # FindInitCovPar values (reference fit fixture) and the summary printout
    import json as _json
    with open(os.path.join(HERE, "golden", "golden_fit.json")) as f:
        ref = _json.load(f)["rtest_dense_exponential"]
    np.testing.assert_allclose(gm.get_init_cov_pars(), ref["init_cov_pars"], rtol=1e-12)
    gm.summary(std_err=True)


@pytest.mark.parametrize("name", ["latent500_bernoulli_m20", "latent500_gaussian_m20"])
def test_fit_matches_reference_latent(golden_fit, name):
    case = golden_fit[name]
    X, Y = _data(case)
    gm = _model(case, X)
    gm.fit(Y, params=_params(case))
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-4)
    if "aux_pars" in case:
        np.testing.assert_allclose(gm.get_aux_pars()[0], case["aux_pars"], rtol=1e-4)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-6 * abs(case["nll"])
    assert abs(gm.get_num_optim_iter() - case["num_it"]) <= 1


def test_fit_offset_and_refit(golden_fit):
    # a Gaussian offset is subtracted from y (OptimLinRegrCoefCovPar :1176-1183); a second fit
    # starts from the previous estimate (re_model.cpp:1142-1164: cov_pars_initialized_)
    case = golden_fit["rtest_dense_exponential"]
    X, Y = _data(case)
    off = np.linspace(-1., 1., Y.shape[0])
    gm = _model(case, X)
    gm.fit(Y + off, offset=off)
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-6)
    nll1 = gm.get_current_neg_log_likelihood()
    gm.fit(Y)   # restarts at the optimum: stops at a point as good, within the 1e-6 objective tolerance
    assert gm.get_current_neg_log_likelihood() <= nll1 + 1e-6 * abs(nll1)
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-2)


def test_fit_errors():
    X, Y = synthetic.rtest_gaussian_y(100)
    gm = GPModel(gp_coords=X, cov_function="exponential")
    with pytest.raises(GPBoostError, match="not supported"):
        gm.fit(Y, params={"optimizer_cov": "adam"})
    gm = GPModel(gp_coords=X, cov_function="exponential")
    with pytest.raises((GPBoostError, ValueError), match="NaN or Inf"):
        gm.fit(np.where(np.arange(100) == 3, np.nan, Y))
    Xb = synthetic.bench_coords(300)
    gl = GPModel(gp_coords=Xb, cov_function="exponential", gp_approx="vecchia", likelihood="bernoulli_logit",
                 num_neighbors=10)
    with pytest.raises(GPBoostError, match="not supported"):   # covariates: Gaussian likelihood only
        gl.fit(synthetic.bench_bernoulli_y(Xb), X=np.ones((300, 1)))


@pytest.mark.parametrize("name", ["sd_rtest_exponential", "sd_rtest_matern15", "sd_rtest_matern25", "sd_rtest_gaussian",
                                  "sd_synth2000_exponential"])
def test_std_dev_matches_reference(golden_fit, name):
    # GPB_GetCovPar(calc_std_dev = true): CalcStdDevCovPar (re_model_template.h:9775-9789), dense
    case = golden_fit[name]
    X, Y = _data(case)
    gm = _model(case, X)
    gm.neg_log_likelihood(case["cov_pars"], Y)   # sets the parameters GPB_GetCovPar reports
    out = gm.get_cov_pars(std_err=True)
    np.testing.assert_allclose(out[0], case["cov_pars"], rtol=1e-15)
    np.testing.assert_allclose(out[1], case["std_dev"], rtol=1e-8)
    if name == "sd_rtest_exponential":   # test_GPModel_gaussian_process.R:122-124 (TOLERANCE_STRICT)
        assert np.sum(np.abs(out[1] - [0.07943467, 0.25351519, 0.03840236])) < 1e-5


def test_std_dev_after_fit_and_errors(golden_fit):
    case = golden_fit["rtest_dense_exponential"]
    X, Y = _data(case)
    gm = _model(case, X)
    gm.fit(Y)
    out = gm.get_cov_pars(std_err=True)
    np.testing.assert_allclose(out[0], case["cov_pars"], rtol=1e-6)
    assert np.all(np.isfinite(out[1])) and np.all(out[1] > 0)
    # full_scale_vecchia: the reference refuses too (re_model_template.h:1666-1668)
    gv = GPModel(gp_coords=X, cov_function="exponential", gp_approx="full_scale_vecchia", num_ind_points=20,
                 num_neighbors=10)
    gv.neg_log_likelihood([0.1, 1.0, 0.1], Y)
    with pytest.raises(GPBoostError, match="standard deviations"):
        gv.get_cov_pars(std_err=True)


def test_fit_maxit_zero_keeps_initial_values(golden_fit):
    case = golden_fit["rtest_dense_exponential"]
    X, Y = _data(case)
    gm = _model(case, X)
    gm.fit(Y, params={"maxit": 0})
    assert gm.get_num_optim_iter() == 0
    np.testing.assert_allclose(gm.get_cov_pars(), case["init_cov_pars"], rtol=1e-12)


def test_latent_fit_recovers_from_nan_trial(golden_fit, monkeypatch):
    """A NaN in a line-search trial of a latent fit shrinks the step instead of failing the fit
    (likelihoods.h:2929-2933 set the marginal likelihood to NaN, LineSearchBacktracking.h:78
    halves the step on fx != fx). Fault injection: the 2nd latent evaluation (the first trial of
    the first line search) reports NaN; the fit must still reach the reference optimum."""
    case = golden_fit["latent500_bernoulli_m20"]
    X, Y = _data(case)
    gm = _model(case, X)
    monkeypatch.setenv("GPBOOST_AMD_TEST_NAN_EVAL", "2")
    gm.fit(Y, params=_params(case))
    monkeypatch.delenv("GPBOOST_AMD_TEST_NAN_EVAL")
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=2e-2)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-5 * abs(case["nll"])
    # without the tolerance of the optimizer the same NaN is an error (GPB_EvalNegLogLikelihood)
    g2 = _model(case, X)
    monkeypatch.setenv("GPBOOST_AMD_TEST_NAN_EVAL", "1")
    with pytest.raises(GPBoostError, match="NaN or Inf"):
        g2.neg_log_likelihood(case["cov_pars"], Y)


@pytest.fixture(scope="module")
def golden_fit_latent():
    with open(os.path.join(HERE, "golden", "golden_fit_latent.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["latent2000_bernoulli_m30_tight", "latent2000_gaussian_m30_tight",
                                  "latent2000_bernoulli_offset_tight"])
def test_fit_matches_reference_latent_tight(golden_fit_latent, name):
    """Latent fits at cg_delta_conv = 1e-8 (tests/golden/make_golden_fit_latent.py): the objective
    continues from the previous evaluation's Laplace mode as the reference's does
    (likelihoods.h:2782-2789), so the L-BFGS path is the reference's: identical iteration count,
    estimates and objective at the north-star 1e-6 (the reference itself repeats these fits only to
    ~4e-7 across runs, its OpenMP reductions being order-dependent)."""
    case = golden_fit_latent[name]
    X = synthetic.bench_coords(case["n"])
    sp = case["spec"]
    if sp["likelihood"] == "bernoulli_logit":
        Y = synthetic.bench_bernoulli_y(X)
    else:
        Y = synthetic.bench_spatial_gaussian_y(X)
    gm = _model(case, X)
    off = 0.5 * np.sin(3 * X[:, 0]) - 0.3 * X[:, 1] if case["offset"] else None
    gm.fit(Y, params=_params(case), offset=off)
    assert gm.get_num_optim_iter() == case["num_it"], (gm.get_num_optim_iter(), case["num_it"])
    np.testing.assert_allclose(gm.get_init_cov_pars(), case["init_cov_pars"], rtol=1e-12)
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-6)
    if "aux_pars" in case:
        np.testing.assert_allclose(gm.get_aux_pars()[0], case["aux_pars"][0], rtol=1e-6)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-6 * abs(case["nll"])


def test_fit_fixed_covariance_parameters_r_golden():
    """estimate_cov_par_index (test_GPModel_gaussian_process.R:232-250): lbfgs with the range, then the marginal
    variance and the range held at their initial values (init var(y)/2, var(y)/2, mean(dist)/3); estimates with
    standard errors (column-major) and nll at the R test's TOLERANCE_STRICT 1e-5."""
    X, Y = synthetic.rtest_gaussian_y(100)
    D = np.sqrt(((X[:, None, :] - X[None, :, :]) ** 2).sum(-1))
    init = np.array([np.var(Y, ddof=1) / 2, np.var(Y, ddof=1) / 2, D[np.triu_indices(100, 1)].mean() / 3])
    for idx, nll_ref, vals in [
        ([1, 1, 0], 123.4853915, [0.10273152252, 0.08925506562, 1.23337072589, 0.37123039633, 0.17864807736, 0.07351705425]),
        ([1, 0, 0], 127.7832271, [0.4583440607, 0.1476785505, 0.5170731356, 0.2240355344, 0.1786480774, 0.1126220657]),
        ([0, 1, 0], 127.9879294, [0.5170731356, 0.1687492120, 0.6088800134, 0.2602195062, 0.1786480774, 0.1112692786]),
        ([0, 0, 0], 128.132446, None),
    ]:
        gm = GPModel(gp_coords=X, cov_function="exponential")
        # params_loc = DEFAULT_OPTIM_PARAMS (lr_cov 0.1, delta_rel_conv 1e-6) with optimizer_cov "lbfgs"
        gm.fit(Y, params={"optimizer_cov": "lbfgs", "lr_cov": 0.1, "delta_rel_conv": 1e-6, "init_cov_pars": init,
                          "estimate_cov_par_index": idx})
        out = gm.get_cov_pars(std_err=True)
        if vals is not None:
            assert np.sum(np.abs(out.T.reshape(-1) - vals)) < 1e-5, (idx, out)
        assert abs(gm.get_current_neg_log_likelihood() - nll_ref) < 1e-5
        for k in range(3):
            if idx[k] == 0:
                assert abs(out[0, k] - init[k]) < 1e-5
    gm = GPModel(gp_coords=X, cov_function="exponential")
    with pytest.raises(GPBoostError, match="estimate_cov_par_index"):
        gm.fit(Y, params={"optimizer_cov": "nelder_mead", "init_cov_pars": init, "estimate_cov_par_index": [1, 1, 0]})
