"""GPU parity for the dense path (gp_approx="none"): blocked MFMA Cholesky, TRTRI, LAUUM,
fused gradient traces, against the reference fixtures, the R-test goldens and the oracle.
Tolerance: 1e-6 relative (BASELINE.json north_star)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-6


def _close(a, b, rtol=RTOL):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.all(np.abs(a - b) <= rtol * np.maximum(np.abs(b), 1.0))


@pytest.mark.parametrize("name", ["rtest_dense_exponential", "rtest_dense_matern15", "rtest_dense_matern25",
                                  "rtest_dense_gaussian", "synth2000_dense_exp"])
def test_dense_matches_reference(golden, rtest_data, synth2000, name):
    from gpboost_amd import GPModel
    case = golden[name]
    X, Y = rtest_data if case["data"] == "rtest_gaussian" else synth2000
    sp = case["spec"]
    gm = GPModel(gp_coords=X, cov_function=sp["cov_fct"], cov_fct_shape=sp.get("shape", 0.5), gp_approx="none")
    nll = gm.neg_log_likelihood(case["cov_pars"], Y)
    assert abs(nll - case["nll"]) <= RTOL * abs(case["nll"])
    if case.get("r_golden") is not None:
        assert abs(nll - case["r_golden"]) < 1e-5
    nll0, g0, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], Y)
    assert abs(nll0 - case["nll"]) <= RTOL * abs(case["nll"])
    assert _close(g0, case["grad"]), (g0, case["grad"])
    nll1, g1, s2 = gm.neg_log_likelihood_and_grad(case["cov_pars"], None, profile_sigma2=True)
    assert abs(nll1 - case["lbfgs_nll"]) <= RTOL * abs(case["lbfgs_nll"])
    assert _close(g1, case["lbfgs_grad"]), (g1, case["lbfgs_grad"])


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 257, 700])
@pytest.mark.parametrize("cov,shape,ct", [("exponential", 0.5, 0), ("gaussian", 0.5, 3)])
def test_dense_vs_oracle_sizes(n, cov, shape, ct):
    """Ragged sizes around the 64/256 block edges."""
    from gpboost_amd import GPModel, synthetic
    X = synthetic.bench_coords(n)
    Y = synthetic.bench_gaussian_y(n)
    pars = [0.3, 1.2, 0.15]
    gm = GPModel(gp_coords=X, cov_function=cov, cov_fct_shape=shape, gp_approx="none")
    tp = O.transform(ct, pars)
    for mode in (0, 1):
        ref = O.dense_nll_grad(X, Y, ct, tp, mode)
        nll, g, _ = gm.neg_log_likelihood_and_grad(pars, Y, profile_sigma2=bool(mode))
        assert abs(nll - ref["nll"]) <= RTOL * abs(ref["nll"]), (n, mode)
        assert _close(g, ref["grad"]), (n, mode, g, ref["grad"])


def test_dense_vecchia_agree_with_full_neighbours(rtest_data):
    """Vecchia with n-1 neighbours and no reordering is exact (R test :711-716): with m = 64 >= n-1
    for n = 65 both GPU paths must agree."""
    from gpboost_amd import GPModel, synthetic
    n = 65
    X = synthetic.bench_coords(n)
    Y = synthetic.bench_gaussian_y(n)
    a = GPModel(gp_coords=X, cov_function="exponential", gp_approx="none").neg_log_likelihood_and_grad(
        [0.1, 1.0, 0.2], Y)
    b = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=64,
                vecchia_ordering="none").neg_log_likelihood_and_grad([0.1, 1.0, 0.2], Y)
    assert abs(a[0] - b[0]) <= 1e-8 * abs(a[0])
    assert _close(a[1], b[1], 1e-7)


def test_dense_not_positive_definite_fails_loudly():
    from gpboost_amd import GPBoostError, GPModel
    X = np.zeros((10, 2))  # all points identical; with a huge variance the nugget still keeps PD,
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="none")
    nll = gm.neg_log_likelihood([1.0, 1.0, 0.1], np.arange(10.0))
    assert np.isfinite(nll)
    with pytest.raises((GPBoostError, ValueError)):
        gm.neg_log_likelihood([1.0, np.nan, 0.1], np.arange(10.0))


def test_dense_5000_gradient_finite_differences():
    from gpboost_amd import GPModel, synthetic
    n = 5000
    X = synthetic.bench_coords(n)
    Y = synthetic.bench_gaussian_y(n)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="none")
    _, g, _ = gm.neg_log_likelihood_and_grad([0.1, 1.0, 0.1], Y)
    h = 1e-5

    def nll_at(lt):
        s2 = np.exp(lt[0]); v = np.exp(lt[1]) * s2; rho = 1.0 / np.exp(lt[2])
        return gm.neg_log_likelihood([s2, v, rho], None)
    lt0 = np.array([np.log(0.1), np.log(10.0), np.log(10.0)])
    fd = [(nll_at(lt0 + h * e) - nll_at(lt0 - h * e)) / (2 * h) for e in np.eye(3)]
    np.testing.assert_allclose(g, fd, rtol=1e-5, atol=1e-3)


def _dense_big_cases():
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_dense_big.json")
    return json.load(open(p)) if os.path.exists(p) else {}


@pytest.mark.parametrize("name", sorted(_dense_big_cases()))
def test_dense_big_matches_reference(name):
    """Parity where the fast dense paths run (BASELINE config 2): at n = 8192 / 20000 the trailing
    updates have >= 512 output tiles of 128, so gemm_f64_big_kernel and the two-stream lookahead
    POTRF / TRTRI / LAUUM are what is checked against the reference (tests/golden/
    make_golden_dense_big.py), in both evaluation modes, at the north-star 1e-6."""
    from gpboost_amd import GPModel, synthetic
    case = _dense_big_cases()[name]
    n = case["n"]
    X = synthetic.bench_coords(n)
    Y = synthetic.bench_gaussian_y(n)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="none")
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], Y)
    assert abs(nll - case["nll"]) <= RTOL * abs(case["nll"]), (nll, case["nll"])
    assert _close(g, case["grad"]), (g, case["grad"])
    nll1, g1, s2 = gm.neg_log_likelihood_and_grad(case["cov_pars"], None, profile_sigma2=True)
    assert abs(nll1 - case["lbfgs_nll"]) <= RTOL * abs(case["lbfgs_nll"]), (nll1, case["lbfgs_nll"])
    assert _close(g1, case["lbfgs_grad"]), (g1, case["lbfgs_grad"])
    assert abs(s2 - case["lbfgs_sigma2"]) <= RTOL * case["lbfgs_sigma2"]
