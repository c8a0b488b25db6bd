"""GPU parity for latent Vecchia models with REPEATED coordinates against the reference itself.

Reference: with duplicate locations the reference runs the latent GP on the unique locations with
an incidence matrix Z (Vecchia_utils.cpp:1121-1139; RECompGP on unique coordinates, re_comp.h:
845-870; only_one_GP_calculations_on_RE_scale_): unique points in order of first appearance in the
shuffled observation order (DetermineUniqueDuplicateCoordsFast, GP_utils.cpp:451-536), the Vecchia
structure over them, and the likelihood's derivative, information and third derivative summed
over each location's observations (Z^T d1, Z^T W Z, Z^T dW) at mode_u + F_i. Fixtures:
tests/golden/golden_latent_dup.json (make_golden_latent_dup.py runs oracle/_ref/ref_harness).

Tolerance: 1e-6 relative (north_star) on nll and gradient, as tests/test_gpu_latent.py; the
cg_delta_conv = 1e-10 cases agree far tighter.
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPBoostError, GPModel, synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
RTOL = 1e-6


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(HERE, "golden", "golden_latent_dup.json")) as f:
        return json.load(f)


def _data(case):
    if case["kind"] == "repeated":
        X = synthetic.repeated_coords(case["n"], case["nu"])
    else:
        X = synthetic.cycled_coords(case["n"])
    lik = case["lik"]
    y = synthetic.bench_bernoulli_y(X) if lik == "bernoulli_logit" else synthetic.bench_gaussian_y(case["n"])
    fe = 0.3 * np.sin(3.0 * X[:, 0]) if case["fe"] else None
    return X, y, fe


def _model(case, X):
    sp = case["spec"]
    gm = GPModel(gp_coords=X, likelihood=case["lik"], cov_function="exponential", gp_approx=sp["gp_approx"],
                 num_neighbors=int(sp["num_neighbors"]), vecchia_ordering="random",
                 matrix_inversion_method="iterative", seed=0)
    params = dict(num_rand_vec_trace=int(sp["num_rand_vec_trace"]), cg_delta_conv=float(sp["cg_delta_conv"]))
    if "aux_pars" in sp:
        params["init_aux_pars"] = [float(sp["aux_pars"])]
    gm.set_optim_params(params)
    return gm


@pytest.mark.parametrize("name", ["bern_rep_n2000_tight", "bern_rep_n2000_default", "bern_rep_n2000_fe_tight",
                                  "gauss_rep_n2000_tight", "gauss_rep_n3000_m10_t20_tight",
                                  "bern_cycled_n100k_tight"])
def test_latent_repeated_coordinates_match_reference(golden, name):
    if name not in golden:
        pytest.skip("fixture not generated (make_golden_latent_dup.py --big)")
    case = golden[name]
    X, y, fe = _data(case)
    assert len(np.unique(X, axis=0)) == case["n_unique"] < case["n"]
    gm = _model(case, X)
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y, fixed_effects=fe)
    assert abs(nll - case["nll"]) <= RTOL * abs(case["nll"]), (nll, case["nll"])
    ref = np.asarray(case["grad"])
    np.testing.assert_allclose(g, ref, rtol=RTOL, atol=RTOL * np.abs(ref).max())
    assert abs(gm.neg_log_likelihood(case["cov_pars"], y, fixed_effects=fe) - nll) <= 1e-12 * abs(nll)


def test_cycled_100k_default_within_reference_sensitivity(golden):
    # n = 100k on the round-1/2 cycling-LCG coordinates (20318 locations), default cg_delta_conv = 1e-2:
    # six Newton steps each solved to an absolute residual of 1e-2 — the gradient is rounding-limited
    # as for config 5 (tests/test_gpu_latent.py). Bound: twice the reference's own spread under
    # 1e-14 relative parameter perturbations (make_golden_latent_dup.py --big); nll at 1e-6.
    if "bern_cycled_n100k_sensitivity" not in golden:
        pytest.skip("fixture not generated (make_golden_latent_dup.py --big)")
    case = golden["bern_cycled_n100k_default"]
    runs = golden["bern_cycled_n100k_sensitivity"]["runs"]
    ref = np.asarray(case["grad"])
    spread = np.max([np.abs(np.asarray(r["grad"]) - ref) for r in runs], axis=0)
    X, y, fe = _data(case)
    gm = _model(case, X)
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= RTOL * abs(case["nll"]), (nll, case["nll"])
    assert np.all(np.abs(g - ref) <= 2 * spread), (g, ref, spread)


def test_latent_repeated_coordinates_mode_per_observation():
    # the training-data prediction of a latent model is the posterior mode Z m: equal at equal coordinates
    X = synthetic.repeated_coords(1500, 400)
    y = synthetic.bench_bernoulli_y(X)
    gm = GPModel(gp_coords=X, likelihood="bernoulli_logit", gp_approx="vecchia", num_neighbors=15,
                 matrix_inversion_method="iterative")
    gm.neg_log_likelihood([1.0, 0.1], y)
    m = gm.predict_training_data_random_effects()
    _, inv = np.unique(X, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    for u in range(inv.max() + 1):
        v = m[inv == u]
        assert np.all(v == v[0])
    with pytest.raises(GPBoostError, match="repeated coordinates"):
        gm.calc_gradient_f(fixed_effects=np.zeros(1500))
    with pytest.raises(GPBoostError, match="repeated coordinates"):
        gm.latent_vecchia_factor([1.0, 0.1])


def test_latent_repeated_coordinates_fit_runs():
    X = synthetic.repeated_coords(2000, 700)
    y = synthetic.bench_bernoulli_y(X)
    gm = GPModel(gp_coords=X, likelihood="bernoulli_logit", gp_approx="vecchia", num_neighbors=20,
                 matrix_inversion_method="iterative")
    gm.fit(y)
    cp = gm.get_cov_pars()
    assert np.all(np.isfinite(cp)) and np.all(cp > 0)
