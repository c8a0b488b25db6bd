"""Pins the full-scale Vecchia (VIF) CPU restatement (oracle/vif_oracle.py + oracle.vif_inducing_points) to the
reference's own outputs (tests/golden/golden_vif.json, make_golden_vif.py): the ordering and the inducing
points bit for bit, the neighbour lists, the nll and gradient with the nugget as a parameter and profiled,
log det Psi and y^T Psi^-1 y. CPU only. Tolerances: nll / pieces 1e-10, gradient 1e-8 (the dense oracle and
the reference's Woodbury formulas are different algebra; observed ~1e-14)."""
import json
import os

import numpy as np
import pytest

from gpboost_amd import synthetic
from oracle import oracle as O
from oracle.vif_oracle import vif_nll_grad

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_vif.json")) as _f:
    GOLDEN = json.load(_f)


def setup_case(case):
    sp = case["spec"]
    n = case["n"]
    X = synthetic.bench_coords(n)
    y = synthetic.bench_spatial_gaussian_y(X)
    perm, Z, _ = O.vif_inducing_points(X, case["m"], sp["ind_points_selection"], sp["seed"], sp["ordering"] == "random")
    xv = X[perm]
    nb = O.find_neighbors(xv, min(case["num_neighbors"], n - 1))
    ct = O.cov_code(sp["cov_fct"], float(sp["shape"]))
    return X, y, perm, Z, xv, nb, ct


@pytest.mark.parametrize("name", [k for k in GOLDEN if k.startswith("vif_") and GOLDEN[k]["n"] <= 3000])
def test_oracle_vif_matches_reference(name):
    case = GOLDEN[name]
    X, y, perm, Z, xv, nb, ct = setup_case(case)
    np.testing.assert_array_equal(perm, case["perm"])
    np.testing.assert_array_equal(Z.ravel(), case["ind_points"])
    for i, row in enumerate(case["neighbors"]):
        assert nb[i, :len(row)].tolist() == row
    tr = O.transform(ct, case["cov_pars"])
    o = vif_nll_grad(xv, y[perm], nb, Z, ct, tr, mode=0)
    assert abs(o["nll"] - case["nll"]) <= 1e-10 * abs(case["nll"])
    assert abs(o["logdet"] - case["log_det_Psi"]) <= 1e-10 * abs(case["log_det_Psi"])
    assert abs(o["q"] - case["yTPsiInvy"]) <= 1e-10 * abs(case["yTPsiInvy"])
    np.testing.assert_allclose(o["grad"], case["grad"], rtol=1e-8, atol=1e-8 * np.abs(case["grad"]).max())
    p = vif_nll_grad(xv, y[perm], nb, Z, ct, tr, mode=1)
    assert abs(p["nll"] - case["nll_profiled"]) <= 1e-10 * abs(case["nll_profiled"])
    np.testing.assert_allclose(p["grad"], case["grad_profiled"], rtol=1e-8)
