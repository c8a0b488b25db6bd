"""GPU parity for grouped (crossed) random effects — BASELINE config 4's expressible proxy
 — against the reference itself.

Reference path: GPB_CreateREModel with re_group_data (re_model_template.h:246-273, RECompGroup
re_comp.h:245-271) -> REModelTemplate<sp_mat_rm_t, chol_sp_mat_rm_t> with the Woodbury identity:
y^T Psi^-1 y and log|Psi| from A = Sigma^-1 + Z^T Z (re_model_template.h:2778-2872, 8965-9005); K >= 2
"iterative" (the default there): SSOR-PCG (CGRandomEffectsVec, CG_utils.cpp:1100-1234), stochastic
Lanczos quadrature (CGTridiagRandomEffects :1236-1414, LogDetStochTridiag :988-1004) and the
stochastic-trace gradient with the SSOR control variate (:2304-2387, CalcOptimalC :1006-1022);
K == 1: the closed-form diagonal branch; K >= 2 "cholesky": the dense M x M factor on the MFMA POTRF (1e-10 nll,
1e-8 gradient: the reference's sparse factor and trace subtraction vs the dense inverse diagonal). Fixtures: tests/golden/golden_grouped.json
(make_golden_grouped.py runs oracle/_ref/ref_harness_grouped, the reference compiled from its
sources).

Tolerances. The probe vectors are the reference's own draws (same mt19937 seeds), so the SLQ and
trace estimates are the same estimators on the same samples: at cg_delta_conv = 1e-10 both sides
run the same Krylov iterations and differ only by summation-order rounding (nll 1e-10 relative,
gradient 1e-6 relative = north_star). At the default cg_delta_conv = 1e-2 the PCG stops after a
handful of iterations whose count both sides share; the remaining difference is rounding of a
truncated solve (same bounds unless a stopping test flips, which these fixtures do not hit). K == 1
is a closed form (1e-10).
"""
import ctypes
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPBoostError, GPModel, synthetic
from gpboost_amd.basic import _dp, _safe_call, lib

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
EVAL_CASES = ["k1_n5000_cholesky", "k2_n20000_tight", "k2_n20000_default", "k3_n20000_tight", "k2_n20000_t20_tight",
              "k2_n20000_cholesky", "k3_n20000_cholesky", "k2_n3000_cholesky_small"]


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(HERE, "golden", "golden_grouped.json")) as f:
        return json.load(f)


def _data(case):
    g = synthetic.bench_groups(case["n"], tuple(case["levels"]))
    return g, synthetic.bench_grouped_y(g)


def _model(case, g):
    o = case["opts"]
    gm = GPModel(group_data=g, matrix_inversion_method=o.get("matrix_inversion_method", "default"))
    params = {}
    if "cg_delta_conv" in o:
        params["cg_delta_conv"] = float(o["cg_delta_conv"])
    if "num_rand_vec_trace" in o:
        params["num_rand_vec_trace"] = int(o["num_rand_vec_trace"])
    if "seed_rand_vec_trace" in o:
        params["seed_rand_vec_trace"] = int(o["seed_rand_vec_trace"])
    gm.set_optim_params(params)
    return gm


@pytest.mark.parametrize("name", EVAL_CASES)
def test_grouped_nll_and_grad_match_reference(golden, name):
    case = golden[name]
    g, y = _data(case)
    gm = _model(case, g)
    cp = np.array(case["cov_pars"])
    nll = gm.neg_log_likelihood(cp, y)
    assert abs(nll - case["nll"]) <= 1e-10 * abs(case["nll"]), (nll, case["nll"])
    nll2, grad, _ = gm.neg_log_likelihood_and_grad(cp, y)
    assert abs(nll2 - case["nll"]) <= 1e-10 * abs(case["nll"])
    np.testing.assert_allclose(grad, case["grad"], rtol=1e-6, atol=1e-6 * np.abs(case["grad"]).max())
    # the L-BFGS unit: sigma^2 profiled out
    nllp, gradp, s2 = gm.neg_log_likelihood_and_grad(cp, y, profile_sigma2=True)
    assert abs(nllp - case["lbfgs_nll"]) <= 1e-10 * abs(case["lbfgs_nll"])
    assert abs(s2 - case["lbfgs_sigma2"]) <= 1e-10 * abs(case["lbfgs_sigma2"])
    np.testing.assert_allclose(gradp, case["lbfgs_grad"], rtol=1e-6, atol=1e-6 * np.abs(case["lbfgs_grad"]).max())


@pytest.mark.parametrize("name", ["fit_k1_n5000", "fit_k2_n20000_tight", "fit_k2_n20000_default",
                                  "fit_k2_n20000_cholesky", "fit_k3_n20000_cholesky"])
def test_grouped_fit_matches_reference(golden, name):
    case = golden[name]
    g, y = _data(case)
    gm = _model(case, g)
    gm.fit(y)
    np.testing.assert_allclose(gm.get_init_cov_pars(), case["init_cov_pars"], rtol=1e-12)
    assert gm.get_num_optim_iter() == case["num_it"]
    np.testing.assert_allclose(gm.get_cov_pars(), case["cov_pars"], rtol=1e-6)
    assert abs(gm.get_current_neg_log_likelihood() - case["nll"]) <= 1e-9 * abs(case["nll"])
    assert gm.cov_par_names() == ["Error_term"] + [f"Group_{k + 1}" for k in range(len(case["levels"]))]


def test_grouped_api_names_and_errors():
    g = synthetic.bench_groups(3000, (60, 9))
    y = synthetic.bench_grouped_y(g)
    gm = GPModel(group_data=g)   # default: iterative with SSOR for K >= 2
    p = gm.get_optim_params()
    assert p["optimizer_cov"] == "lbfgs" and p["cg_preconditioner_type"] == "ssor"
    assert gm.num_cov_pars == 3
    gm.neg_log_likelihood([1.0, 0.5, 0.5], y)
    np.testing.assert_array_equal(gm.get_response_data(), y)
    with pytest.raises(GPBoostError, match="single-level grouped"):
        GPModel(group_data=g[:, :1], matrix_inversion_method="iterative")
    with pytest.raises(GPBoostError, match="not supported"):
        gm.set_optim_params({"cg_preconditioner_type": "incomplete_cholesky"})
    with pytest.raises(GPBoostError, match="grouped random effects"):
        gm.vecchia_structure()


def test_grouped_string_labels_equal_integer_labels():
    # labels are strings in the C API (order of first appearance defines the level index)
    g = synthetic.bench_groups(4000, (80, 11))
    y = synthetic.bench_grouped_y(g)
    names = np.array([f"city_{v}" for v in g[:, 0]], dtype=object)
    gs = np.column_stack([names, g[:, 1].astype(str)])
    a = GPModel(group_data=g).neg_log_likelihood_and_grad([1.0, 0.7, 0.3], y)
    b = GPModel(group_data=gs).neg_log_likelihood_and_grad([1.0, 0.7, 0.3], y)
    assert a[0] == b[0]
    np.testing.assert_array_equal(a[1], b[1])


def test_grouped_config4_size_matches_reference(golden):
    # BASELINE config 4 size: n = 500000, 5000 + 500 levels (make_golden_grouped.py --big)
    for name in ("k2_n500000_default", "k2_n500000_tight"):
        if name not in golden:
            pytest.skip("config-4 fixtures not generated")
        case = golden[name]
        g, y = _data(case)
        gm = _model(case, g)
        cp = np.array(case["cov_pars"])
        nll, grad, _ = gm.neg_log_likelihood_and_grad(cp, y)
        assert abs(nll - case["nll"]) <= 1e-10 * abs(case["nll"]), (name, nll, case["nll"])
        np.testing.assert_allclose(grad, case["grad"], rtol=1e-6, atol=1e-6 * np.abs(case["grad"]).max())


def _levels_of(g):
    """Per effect: the level index of every observation (order of first appearance)."""
    out = []
    for k in range(g.shape[1]):
        _, first, inv = np.unique(g[:, k], return_index=True, return_inverse=True)
        order = np.argsort(first)
        rank = np.empty_like(order)
        rank[order] = np.arange(order.size)
        out.append(rank[inv])
    return out


@pytest.mark.parametrize("name", ["pred_train_k1_n5000", "pred_train_k2_n20000_tight",
                                  "pred_train_k3_n20000_default", "pred_train_k2_n20000_cholesky",
                                  "pred_train_k3_n20000_cholesky"])
def test_grouped_training_data_random_effects_match_reference(golden, name):
    # PredictTrainingDataRandomEffects, grouped branch (re_model_template.h:4065-4167): the posterior
    # mean tau_k Z_k^T Psi^-1 y of each observation's level; K == 1 also its variance (closed form)
    case = golden[name]
    g, y = _data(case)
    gm = _model(case, g)
    K = g.shape[1]
    cp = np.array(case["cov_pars"])
    gm.neg_log_likelihood(cp, y)   # sets y and the parameters
    want_var = "var_levels" in case
    out = np.zeros((2 if want_var else 1) * K * case["n"])
    _safe_call(lib().GPB_PredictREModelTrainingDataRandomEffects(gm.handle, _dp(cp), None, _dp(out), None,
                                                                 ctypes.c_bool(want_var)))
    lev = _levels_of(g)
    mean = out[:K * case["n"]].reshape(K, -1)
    for k in range(K):
        ref = np.asarray(case["mean_levels"][k])[lev[k]]
        # tight: rounding of the PCG iterates (1e-9 of the largest mean); default tolerance: the same
        # truncated PCG on both sides
        np.testing.assert_allclose(mean[k], ref, rtol=0, atol=1e-8 * np.abs(ref).max())
        if want_var:
            v = out[K * case["n"]:].reshape(K, -1)[k]
            # K == 1 closed form 1e-12; K >= 2 cholesky: diag(A^-1) from the dense inverse factor
            np.testing.assert_allclose(v, np.asarray(case["var_levels"][k])[lev[k]], rtol=1e-12 if K == 1 else 1e-9)


def test_grouped_predict_new_and_seen_levels():
    g = synthetic.bench_groups(6000, (120, 15))
    y = synthetic.bench_grouped_y(g)
    gm = GPModel(group_data=g)
    cp = [1.0, 0.8, 0.3]
    gm.neg_log_likelihood(cp, y)
    tr = gm.predict_training_data_random_effects()          # (n, 2): per-effect posterior means
    assert tr.shape == (6000, 2)
    # at the training labels the predictive mean is the sum of the effects' posterior means
    p = gm.predict(group_data_pred=g[:500], cov_pars=cp, predict_var=False)
    np.testing.assert_allclose(p["mu"], tr[:500].sum(axis=1), rtol=0, atol=1e-12 * np.abs(tr).max())
    # an unseen level contributes 0; an offset is added
    gn = np.array([[10_000, g[0, 1]], [g[1, 0], 99_999], [77_777, 88_888]])
    p = gm.predict(group_data_pred=gn, cov_pars=cp, offset_pred=np.array([1., 2., 3.]))
    np.testing.assert_allclose(p["mu"], [tr[0, 1] + 1., tr[1, 0] + 2., 3.], rtol=0, atol=1e-12 * np.abs(tr).max())
    with pytest.raises(GPBoostError, match="predictive"):   # iterative: the reference's simulation, refused
        gm.predict(group_data_pred=g[:5], cov_pars=cp, predict_var=True)
    with pytest.raises(GPBoostError, match="not implemented for matrix_inversion_method_ == 'iterative'"):
        gm.predict_training_data_random_effects(predict_var=True)


def test_grouped_predict_saved_data():
    """set_prediction_data(group_data_pred=...) -> predict(use_saved_data=True) (reference basic.py
    6095-6190, re_model_template.h:3081-3085, 3168-3206): the same means as passing the labels."""
    g = synthetic.bench_groups(6000, (120, 15))
    y = synthetic.bench_grouped_y(g)
    gm = GPModel(group_data=g)
    cp = [1.0, 0.8, 0.3]
    gm.neg_log_likelihood(cp, y)
    gn = np.vstack([g[:40], [[10_000, g[0, 1]], [77_777, 88_888]]])
    direct = gm.predict(group_data_pred=gn, cov_pars=cp)
    gm.set_prediction_data(group_data_pred=gn)
    saved = gm.predict(cov_pars=cp, use_saved_data=True)
    np.testing.assert_array_equal(saved["mu"], direct["mu"])


GOLDEN_PRED = os.path.join(HERE, "golden", "golden_grouped_pred.json")


@pytest.mark.parametrize("name", ["gp_k1_var_resp", "gp_k1_cov", "gp_k2_var_resp", "gp_k2_var", "gp_k2_cov_resp",
                                  "gp_k3_var", "gp_k3_cov"])
def test_grouped_predictive_variances_match_reference(name):
    """Predictive variances / covariance matrices at new labels (seen levels, repeated new labels, mixes),
    matrix_inversion_method = "cholesky" (CalcPred, re_model_template.h:10350-10358, 10510-10522): the
    reference's sparse triangular solves vs e_p^T A^-1 e_q from the dense inverse factor: 1e-9."""
    with open(GOLDEN_PRED) as f:
        case = json.load(f)[name]
    g = synthetic.bench_groups(case["n"], tuple(case["levels"]))
    y = synthetic.bench_grouped_y(g)
    gm = GPModel(group_data=g, matrix_inversion_method="cholesky")
    cp = np.array(case["cov_pars"])
    want_cov = "cov" in case
    p = gm.predict(y=y, group_data_pred=np.array(case["labels"]), cov_pars=cp, predict_var=not want_cov,
                   predict_cov_mat=want_cov, predict_response=case["response"])
    np.testing.assert_allclose(p["mu"], case["mean"], rtol=0, atol=1e-10 * np.abs(case["mean"]).max())
    if want_cov:
        ref = np.asarray(case["cov"]).reshape(case["npred"], case["npred"])
        np.testing.assert_allclose(p["cov"], ref, rtol=1e-9, atol=1e-12 * np.abs(ref).max())
    else:
        np.testing.assert_allclose(p["var"], case["var"], rtol=1e-9)


@pytest.mark.parametrize("name", ["sdg_k1_n5000", "sdg_k2_n20000", "sdg_k3_n20000", "sdg_k2_n3000_small"])
def test_grouped_std_dev_matches_reference(name):
    """get_cov_pars(std_err=True), cholesky: CalcFisherInformation_Only_Grouped_REs_Woodbury
    (re_model_template.h:9559-9651) restated through B = S^1/2 A^-1 S^1/2 on the GPU (csrc/grouped.h):
    1e-8 against the reference (its sparse solves vs the dense inverse)."""
    with open(os.path.join(HERE, "golden", "golden_grouped_sd.json")) as f:
        case = json.load(f)[name]
    g = synthetic.bench_groups(case["n"], tuple(case["levels"]))
    y = synthetic.bench_grouped_y(g)
    gm = GPModel(group_data=g, matrix_inversion_method="cholesky")
    assert gm.can_calculate_standard_errors_cov_pars()
    gm.neg_log_likelihood(case["cov_pars"], y)
    out = gm.get_cov_pars(std_err=True)
    np.testing.assert_allclose(out[1], case["std_dev"], rtol=1e-8)
    gi = GPModel(group_data=g) if g.shape[1] > 1 else None   # iterative: the stochastic estimate is refused
    if gi is not None:
        assert not gi.can_calculate_standard_errors_cov_pars()
        gi.neg_log_likelihood(case["cov_pars"], y)
        with pytest.raises(GPBoostError, match="standard deviations"):
            gi.get_cov_pars(std_err=True)
