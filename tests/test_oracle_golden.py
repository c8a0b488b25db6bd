"""CPU: pin the oracle (oracle/gp_oracle.cpp) to the reference.

(a) golden numbers hard-coded in the reference's own R tests
    (R-package/tests/testthat/test_GPModel_gaussian_process.R:81, 97, 108, 711-716, 744-749),
(b) fixtures produced by the reference itself (oracle/_ref/ref_harness built from
    /root/reference; tests/golden/make_golden.py): nll and gradient in both evaluation
    modes, the Vecchia permutation, neighbour lists (bit-exact), B and D^-1.
"""
import numpy as np
import pytest

from oracle import oracle as O

R_TOL = 1e-5           # TOLERANCE_STRICT of the R tests
REL = 1e-9             # oracle vs reference fixtures (same math, different summation order)


def _data(case, rtest_data, synth2000):
    if case["data"] == "rtest_gaussian":
        return rtest_data
    if case["n"] == 2000:
        return synth2000
    from gpboost_amd import synthetic
    return synthetic.bench_coords(case["n"]), synthetic.bench_gaussian_y(case["n"])


def _oracle_eval(case, X, Y, mode):
    sp = case["spec"]
    ct = O.cov_code(sp["cov_fct"], sp.get("shape", 0.5))
    tp = O.transform(ct, case["cov_pars"])
    if sp["gp_approx"] == "vecchia":
        perm, xv, nb = O.vecchia_setup(X, sp["num_neighbors"], 0, sp["ordering"] == "random")
        return O.vecchia_nll_grad(xv, Y[perm], nb, ct, tp, mode)
    return O.dense_nll_grad(X, Y, ct, tp, mode)


def test_r_goldens(golden, rtest_data):
    X, Y = rtest_data
    n_checked = 0
    for name, case in golden.items():
        if case.get("r_golden") is None:
            continue
        r = _oracle_eval(case, X, Y, 0)
        assert abs(r["nll"] - case["r_golden"]) < R_TOL, name
        n_checked += 1
    assert n_checked == 5


@pytest.mark.parametrize("mode", [0, 1])
def test_reference_fixtures(golden, rtest_data, synth2000, mode):
    for name, case in golden.items():
        if case["n"] > 2000:
            continue
        X, Y = _data(case, rtest_data, synth2000)
        r = _oracle_eval(case, X, Y, mode)
        nll_ref = case["nll"] if mode == 0 else case["lbfgs_nll"]
        g_ref = np.array(case["grad"] if mode == 0 else case["lbfgs_grad"])
        assert abs(r["nll"] - nll_ref) <= REL * abs(nll_ref), name
        np.testing.assert_allclose(r["grad"], g_ref, rtol=1e-8, atol=1e-8 * np.abs(g_ref).max(), err_msg=name)
        if mode == 1:
            assert abs(r["sigma2"] - case["lbfgs_sigma2"]) <= REL * case["lbfgs_sigma2"], name


def test_vecchia_structure_bit_exact(golden_arrays, synth2000):
    X, _ = synth2000
    perm, xv, nb = O.vecchia_setup(X, 30, 0, True)
    assert np.array_equal(perm, golden_arrays["synth2000_perm"])
    assert np.array_equal(nb, golden_arrays["synth2000_neighbors"])


def test_vecchia_structure_bit_exact_20000(golden_arrays):
    from gpboost_amd import synthetic
    X = synthetic.bench_coords(20000)
    perm, xv, nb = O.vecchia_setup(X, 30, 0, True)
    assert np.array_equal(perm, golden_arrays["synth20000_perm"])
    assert np.array_equal(nb, golden_arrays["synth20000_neighbors"])


def test_vecchia_factor_matches_reference(golden_arrays, synth2000):
    X, Y = synth2000
    perm, xv, nb = O.vecchia_setup(X, 30, 0, True)
    tp = O.transform(0, [0.1, 1.0, 0.1])
    r = O.vecchia_nll_grad(xv, Y[perm], nb, 0, tp, 0, want_factor=True)
    np.testing.assert_allclose(r["Dinv"], golden_arrays["synth2000_Dinv"], rtol=1e-10)
    np.testing.assert_allclose(r["B"], golden_arrays["synth2000_B"], rtol=1e-9, atol=1e-12)


def test_partials_sum_to_whole(synth2000):
    """Row-block partial sums add up to the full-range sums (reduction contract)."""
    X, Y = synth2000
    perm, xv, nb = O.vecchia_setup(X, 30, 0, True)
    tp = O.transform(0, [0.1, 1.0, 0.1])
    full = O.vecchia_partials(xv, Y[perm], nb, 0, tp, 0, 2000)
    parts = sum(O.vecchia_partials(xv, Y[perm], nb, 0, tp, a, b) for a, b in [(0, 7), (7, 999), (999, 2000)])
    np.testing.assert_allclose(parts, full, rtol=1e-12)


def test_oracle_vecchia_prediction_matches_r_golden():
    """Exact Gaussian Vecchia prediction, vecchia_pred_type = "order_obs_first_cond_obs_only",
    30 neighbours, vecchia_ordering = "none", at the fitted parameters the R test prints
    (test_GPModel_gaussian_process.R:912-931: cov_pars_vecchia (0.03297349, 1.07691542,
    0.11378505) -> expected_mu_vecchia, expected_cov_vecchia diagonal; predict_response = TRUE).
    The parameters are printed to 8 digits, so the golden pins the oracle to ~1e-7."""
    from gpboost_amd import synthetic
    coords, y = synthetic.rtest_gaussian_y(100)
    xp = np.array([[0.1, 0.9], [0.10001, 0.90001], [0.7, 0.55]])
    tp = O.transform(0, [0.03297349, 1.07691542, 0.11378505])
    mu, var, nb = O.vecchia_predict(coords, y, xp, 30, 0, tp, predict_response=True)
    assert np.abs(mu - np.array([0.06968068, 0.06967750, 0.44208925])).sum() < 2e-6
    assert np.abs(var - np.array([0.6214955, 0.6215069, 0.4199531])).sum() < 2e-6
    # latent process: the nugget variance (sigma2) removed
    mu0, var0, _ = O.vecchia_predict(coords, y, xp, 30, 0, tp, predict_response=False)
    np.testing.assert_array_equal(mu0, mu)
    np.testing.assert_allclose(var0, var - 0.03297349, rtol=0, atol=1e-12)
