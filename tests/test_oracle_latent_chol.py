"""The numpy restatement of the latent Vecchia Cholesky path (oracle/latent_chol_oracle.py) against the reference's
own fixtures (tests/golden/golden_latent_chol.json, make_golden_latent_chol.py): nll at 1e-10, gradient at 1e-7
(dense algebra on both sides, different summation order), the gradient wrt F, and the R tests' values."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from oracle.latent_chol_oracle import LatentCholOracle

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


def _oracle(case, fe=None):
    sp = case["spec"]
    X, y = _data(case["data"], case["n"])
    ct = O.cov_code(sp["cov_fct"], float(sp["shape"]))
    m = min(int(sp["num_neighbors"]), case["n"] - 1)
    perm, xv, nb = O.vecchia_setup(X, m, 0, sp["ordering"] == "random")
    aux = case.get("aux") or 1.0
    F = None if fe is None else fe(X)[perm]
    o = LatentCholOracle(xv, y[perm], nb, ct, O.transform_latent(ct, case["cov_pars"]), sp["likelihood"], aux=aux,
                         fixed_effects=F)
    return o, perm


@pytest.mark.parametrize("name", [k for k in GOLDEN if GOLDEN[k]["kind"] == "eval" and GOLDEN[k]["n"] <= 2000])
def test_oracle_latent_chol_matches_reference(name):
    case = GOLDEN[name]
    o, _ = _oracle(case)
    assert abs(o.nll - case["nll"]) <= 1e-10 * abs(case["nll"]), (o.nll, case["nll"])
    g, _ = o.grad()
    np.testing.assert_allclose(g, case["grad"], rtol=1e-7, atol=1e-9 * abs(case["nll"]))
    if "r_expected_nll" in case:
        assert abs(o.nll - case["r_expected_nll"]) < 1e-5


def test_oracle_latent_chol_gradient_wrt_fixed_effects():
    case = GOLDEN["gradf_pois_m20_n1000"]
    o, perm = _oracle(case, fe=lambda X: 0.3 * np.sin(3.0 * X[:, 0]) - 0.2)
    assert abs(o.nll - case["nll"]) <= 1e-10 * abs(case["nll"])
    g, gf = o.grad()
    np.testing.assert_allclose(g, case["grad"], rtol=1e-7)
    out = np.empty_like(gf)
    out[perm] = gf
    np.testing.assert_allclose(out, case["grad_f"], rtol=1e-8, atol=1e-10)
