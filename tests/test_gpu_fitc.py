"""GPU parity for the FITC approximation (gp_approx = "fitc", Gaussian likelihood) through the C ABI.

Reference: CreateREComponentsFITC_FSA (re_model_template.h:6931-7073; kmeans++ GP_utils.cpp:203-295),
CalcSigmaComps (:7341-7378), CalcCovFactorFITC_FSA (:8823-8863), CalcYAux (:8898-8908), log det
(:2698-2714), CalcGradPars_FITC_FSA_GaussLikelihood_Cluster_i (:1985-2232). Fixtures:
tests/golden/golden_fitc.json (the reference itself; make_golden_fitc.py), checked against the CPU
oracle in test_oracle_fitc.py.

Tolerances: inducing points bit-exact (kmeans++ seeding on the host with the same std:: draws, Lloyd
iterations on the GPU with the reference's uncontracted distance / mean arithmetic); nll 1e-9 and
gradient 1e-7 relative (fp64 MFMA GEMMs and Woodbury identities vs the reference's Eigen products:
rounding only); fits: the same iteration count, estimates to 1e-6 relative.
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPBoostError, GPModel, synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_fitc.json")) as _f:
    GOLDEN = json.load(_f)
EVAL = [k for k, v in GOLDEN.items() if "lbfgs" in v]
FITS = [k for k in GOLDEN if k.startswith("fit_")]
PREDS = [k for k in GOLDEN if k.startswith("pred_")]


def _data(case):
    X = synthetic.bench_coords(case["n"])
    return X, synthetic.bench_spatial_gaussian_y(X)


def _model(case, X):
    sp = case["spec"]
    return GPModel(gp_coords=X, cov_function=sp["cov_fct"], cov_fct_shape=float(sp.get("shape", 0.5)),
                   gp_approx="fitc", num_ind_points=int(sp["num_ind_points"]),
                   ind_points_selection=sp.get("ind_points_selection", "kmeans++"), seed=int(sp.get("seed", 0)))


@pytest.mark.parametrize("name", EVAL)
def test_fitc_matches_reference(name):
    case = GOLDEN[name]
    X, y = _data(case)
    gm = _model(case, X)
    Z = gm.inducing_points()
    ref_z = np.array(case["ind_points"]).reshape(case["m"], -1)
    assert np.array_equal(Z, ref_z), np.max(np.abs(Z - ref_z))
    for mode, key in ((False, "eval"), (True, "lbfgs")):
        if key not in case:
            continue
        ref = case[key]
        nll, g, s2 = gm.neg_log_likelihood_and_grad(case["cov_pars"], y, profile_sigma2=mode)
        assert abs(nll - ref["nll"]) <= 1e-9 * abs(ref["nll"]), (key, nll, ref["nll"])
        np.testing.assert_allclose(g, ref["grad"], rtol=1e-7, atol=1e-9 * abs(ref["nll"]))
        # sigma^2 = y^T Psi^-1 y / n of the profiled unit: the Gaussian kernel's ill-conditioned K_mm
        # (m = 80) amplifies rounding in the Woodbury solve to ~1e-9
        assert abs(s2 - ref["sigma2"]) <= 1e-8 * abs(ref["sigma2"])


@pytest.mark.parametrize("name", FITS)
def test_fitc_fit_matches_reference(name):
    case = GOLDEN[name]
    X, y = _data(case)
    gm = _model(case, X)
    gm.fit(y)
    # FindInitCovPar on the inducing points (re_model_template.h:4474-4476)
    np.testing.assert_allclose(gm.get_init_cov_pars(), case["init_cov_pars"], rtol=1e-12)
    assert gm.get_num_optim_iter() == case["num_it"]
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-6)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-9 * abs(case["nll"])


def test_fitc_nll_only_equals_grad_eval():
    case = GOLDEN["fitc_exp_n2000_m50"]
    X, y = _data(case)
    gm = _model(case, X)
    nll0 = gm.neg_log_likelihood(case["cov_pars"], y)
    nll1, _, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert nll0 == nll1


def test_fitc_gradient_f_is_psi_inverse_y():
    # GPB_CalcGradientF (Gaussian): Psi^-1 (F - y) / sigma^2 -> its inner product with (F - y) is
    # y^T Psi^-1 y / sigma^2 of the evaluation at the same parameters (yTPsiInvy of the fixture)
    case = GOLDEN["fitc_exp_n2000_m50"]
    X, y = _data(case)
    gm = _model(case, X)
    gm.set_optim_params({"init_cov_pars": case["cov_pars"]})
    g = gm.calc_gradient_f(-y)
    ref = case["eval"]["yTPsiInvy"] / case["cov_pars"][0]
    assert abs(float(np.dot(g, -y)) - ref) <= 1e-9 * abs(ref)


def test_fitc_refusals():
    X = synthetic.bench_coords(500)
    with pytest.raises(GPBoostError, match="iterative"):
        GPModel(gp_coords=X, gp_approx="fitc", num_ind_points=20, matrix_inversion_method="iterative")
    with pytest.raises(GPBoostError, match="more inducing points"):
        GPModel(gp_coords=X, gp_approx="fitc", num_ind_points=600)
    Xd = np.vstack([X, X[:10]])
    with pytest.raises(GPBoostError, match="duplicate"):
        GPModel(gp_coords=Xd, gp_approx="fitc", num_ind_points=20)
    with pytest.raises(GPBoostError, match="cover_tree|not supported"):
        GPModel(gp_coords=X, gp_approx="fitc", num_ind_points=20, ind_points_selection="cover_tree")


@pytest.mark.parametrize("name", PREDS)
def test_fitc_predict_matches_reference(name):
    """CalcPredFITC_FSA (re_model_template.h:10600-10828): means, variances or the covariance matrix at
    new points, and at training coordinates (the FITC diagonal correction, :10643-10691, 10706-10708,
    10799-10826), latent and response scale, against the reference at 1e-9."""
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
    np.testing.assert_allclose(pred["mu"], mu, rtol=1e-9, atol=1e-9 * np.abs(mu).max())
    if want_cov:
        c = np.asarray(case["cov"]).reshape(npred, npred)
        np.testing.assert_allclose(pred["cov"], c, rtol=1e-9, atol=1e-9 * np.abs(c).max())
    else:
        np.testing.assert_allclose(pred["var"], case["var"], rtol=1e-9, atol=1e-12)
