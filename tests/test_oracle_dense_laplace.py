"""Pins the dense Laplace restatement (oracle/dense_laplace_oracle.py: FindModePostRandEffCalcMLLStable,
CalcGradNegMargLikelihoodLaplaceApproxStable, PredictLaplaceApproxStable, likelihoods.h:1843-1960,
3261-3413, 5610-5676) to the reference's fixtures (tests/golden/golden_dense_laplace.json,
make_golden_dense_laplace.py) at 1e-10 (nll) / 1e-8 (gradients, predictions): both are exact dense algebra."""
import json
import os

import numpy as np
import pytest

from conftest import lik_case_data
from gpboost_amd import synthetic
from oracle.dense_laplace_oracle import DenseLaplaceOracle

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_dense_laplace.json")) as _f:
    GOLDEN = json.load(_f)
with open(os.path.join(HERE, "golden", "golden_gamma.json")) as _f:
    GAMMA = json.load(_f)

CT = {("exponential", "0.5"): 0, ("matern", "1.5"): 1, ("matern", "2.5"): 2, ("gaussian", "0.0"): 3}


def _oracle(case, fe=None):
    X, y = lik_case_data(case)
    sp = case["spec"]
    ct = CT[(sp["cov_fct"], sp["shape"])]
    var, rho = case["cov_pars"]
    phi = {0: 1. / rho, 1: np.sqrt(3.) / rho, 2: np.sqrt(5.) / rho, 3: 1. / rho ** 2}[ct]
    return X, DenseLaplaceOracle(X, y, ct, var, phi, sp["likelihood"], fixed_effects=fe)


@pytest.mark.parametrize("name", [k for k in GOLDEN if GOLDEN[k]["kind"] == "eval" and GOLDEN[k]["n"] <= 1000])
def test_oracle_dense_laplace_matches_reference(name):
    case = GOLDEN[name]
    _, o = _oracle(case)
    assert abs(o.nll - case["nll"]) <= 1e-10 * abs(case["nll"])
    g, _ = o.grad()
    np.testing.assert_allclose(g, case["grad"], rtol=1e-8)
    if "r_expected_nll" in case:
        assert abs(o.nll - case["r_expected_nll"]) < 1e-5


@pytest.mark.parametrize("name", [k for k in GOLDEN if GOLDEN[k]["kind"] == "gradf"])
def test_oracle_dense_laplace_gradient_f(name):
    case = GOLDEN[name]
    X, _ = lik_case_data(case)
    _, o = _oracle(case, fe=0.3 * np.sin(3.0 * X[:, 0]) - 0.2)
    assert abs(o.nll - case["nll"]) <= 1e-10 * abs(case["nll"])
    g, gf = o.grad()
    np.testing.assert_allclose(g, case["grad"], rtol=1e-8)
    np.testing.assert_allclose(gf, case["grad_f"], rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("name", [k for k in GOLDEN if GOLDEN[k]["kind"] == "pred" and not GOLDEN[k]["response"]])
def test_oracle_dense_laplace_predict(name):
    case = GOLDEN[name]
    X, o = _oracle(case)
    npred = case["npred"]
    xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    xp[: min(5, npred)] = X[: min(5, npred)]
    want_cov = "cov" in case
    mean, v = o.predict(xp, want_cov)
    np.testing.assert_allclose(mean, case["mean"], rtol=1e-8, atol=1e-10)
    ref = np.asarray(case["cov"]).reshape(npred, npred) if want_cov else np.asarray(case["var"])
    np.testing.assert_allclose(v, ref, rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("name", [k for k in GAMMA if GAMMA[k]["kind"] == "eval" and GAMMA[k]["spec"]["gp_approx"] == "none"])
def test_oracle_dense_laplace_gamma(name):
    """likelihood 'gamma' incl. the shape gradient (golden_gamma.json, make_golden_gamma.py); the R test's nll."""
    case = GAMMA[name]
    X, y = lik_case_data(case)
    sp = case["spec"]
    ct = CT[(sp["cov_fct"], sp["shape"])]
    var, rho = case["cov_pars"]
    phi = {0: 1. / rho, 1: np.sqrt(3.) / rho, 2: np.sqrt(5.) / rho, 3: 1. / rho ** 2}[ct]
    o = DenseLaplaceOracle(X, y, ct, var, phi, "gamma", aux=case["aux"])
    assert abs(o.nll - case["nll"]) <= 1e-10 * abs(case["nll"])
    g, _ = o.grad()
    ref = np.asarray(case["grad"])
    np.testing.assert_allclose(g[: len(ref)], ref, rtol=1e-8)
    if "r_expected_nll" in case:
        assert abs(o.nll - case["r_expected_nll"]) < 1e-5
