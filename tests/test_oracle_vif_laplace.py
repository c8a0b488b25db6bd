"""Pins the full-scale Vecchia Laplace restatement (oracle/vif_laplace_oracle.py) to the reference's own outputs
(tests/golden/golden_vif_laplace.json, make_golden_vif_laplace.py): the ordering, inducing points and neighbour lists,
the latent residual factor's D^-1, the nll and gradient (incl. the gamma shape) and the gradient wrt the fixed
effects (the reference's covariance gradient evaluates its location-dependent terms at mode + F with F in data
order, not in FSVA's model order, re_model_template.h:1859; reproduced, see csrc/vif_laplace.h). CPU only. Tolerances: D^-1 1e-8 (residual variances k - |V|^2 - A.c are formed by cancellation; observed 4e-10), nll 2e-9,
gradient 1e-7 (observed 1e-15 .. 1e-9 / 1e-14 .. 4e-8, the larger values with smooth kernels, cond(M) ~1e5-1e6; the dense oracle and the
reference's sparse / Woodbury formulas are different algebra)."""
import json
import os

import numpy as np
import pytest

from gpboost_amd import synthetic
from oracle import oracle as O
from oracle.vif_laplace_oracle import VifLaplaceOracle

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_vif_laplace.json")) as _f:
    GOLDEN = json.load(_f)


def data(kind, n):
    X = synthetic.bench_coords(n)
    if kind == "bench_gamma":
        return X, synthetic.bench_gamma_y(X)
    if kind == "bench_pois":
        return X, synthetic.bench_poisson_y(X)
    return X, synthetic.bench_bernoulli_y(X)


def setup(case):
    sp = case["spec"]
    X, y = data(case["data"], case["n"])
    perm, Z, _ = O.vif_inducing_points(X, sp["num_ind_points"], sp["ind_points_selection"], sp["seed"], True)
    xv = X[perm]
    nb = O.find_neighbors(xv, min(sp["num_neighbors"], case["n"] - 1))
    ct = O.cov_code(sp["cov_fct"], float(sp["shape"]))
    return X, y, perm, Z, xv, nb, ct


EVALS = [k for k, v in GOLDEN.items() if v["kind"] == "eval" and v["n"] <= 2000]


@pytest.mark.parametrize("name", EVALS)
def test_oracle_vif_laplace_matches_reference(name):
    case = GOLDEN[name]
    sp = case["spec"]
    X, y, perm, Z, xv, nb, ct = setup(case)
    np.testing.assert_array_equal(perm, case["perm"])
    np.testing.assert_array_equal(Z.ravel(), case["ind_points"])
    for i, row in enumerate(case["neighbors"]):
        assert nb[i, :len(row)].tolist() == row
    tr = O.transform_latent(ct, case["cov_pars"])
    aux = case["aux"] if case["aux"] is not None else 1.
    o = VifLaplaceOracle(xv, y[perm], nb, Z, ct, tr[0], tr[1], sp["likelihood"], aux=aux)
    np.testing.assert_allclose(1. / o.D, case["D_inv"], rtol=1e-8)   # residual variances by cancellation
    assert abs(o.nll - case["nll"]) <= 2e-9 * abs(case["nll"])
    g, _ = o.grad()
    ref = np.array(case["grad"])
    np.testing.assert_allclose(g, ref, rtol=1e-7, atol=1e-7 * np.abs(ref).max())


def test_oracle_vif_laplace_grad_f_matches_reference():
    case = GOLDEN["gradf_pois_m30_nn10_n1000"]
    sp = case["spec"]
    X, y, perm, Z, xv, nb, ct = setup(case)
    fe = 0.3 * np.sin(3.0 * X[:, 0]) - 0.2
    tr = O.transform_latent(ct, case["cov_pars"])
    o = VifLaplaceOracle(xv, y[perm], nb, Z, ct, tr[0], tr[1], sp["likelihood"], fixed_effects=fe[perm])
    assert abs(o.nll - case["nll"]) <= 1e-10 * abs(case["nll"])
    # the reference's covariance gradient sees the fixed effects in data order (re_model_template.h:1859)
    g, _ = o.grad(grad_offset=fe)
    np.testing.assert_allclose(g, case["grad"], rtol=1e-8)
    _, gf = o.grad()
    out = np.empty_like(gf)
    out[perm] = gf
    np.testing.assert_allclose(out, case["grad_f"], rtol=1e-8, atol=1e-10)
