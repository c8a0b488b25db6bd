"""The Newton mode-change cap of count likelihoods (CapChangeModeUpdateNewton, likelihoods.h:11800-11810): the
dense restatements (oracle/latent_chol_oracle.py, oracle/vif_laplace_oracle.py) against the reference's own values
for Poisson counts of a few hundred, where the first Newton step from 0 exceeds log(100)
(tests/golden/golden_mode_cap.json, make_golden_mode_cap.py). CPU only."""
import json
import os

import numpy as np

from gpboost_amd import synthetic
from oracle import oracle as O
from oracle.latent_chol_oracle import LatentCholOracle
from oracle.vif_laplace_oracle import VifLaplaceOracle

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_mode_cap.json")) as _f:
    GOLDEN = json.load(_f)


def _data(n):
    X = synthetic.bench_coords(n)
    return X, np.round(300. * np.exp(np.sin(4. * X[:, 0]) * np.cos(3. * X[:, 1])))


def test_oracle_latent_chol_mode_cap_matches_reference():
    case = GOLDEN["vecchia_chol_pois_m20"]
    X, y = _data(case["n"])
    perm = O.vecchia_order(case["n"], 0, True)
    xv = X[perm]
    nb = O.find_neighbors(xv, case["spec"]["num_neighbors"])
    o = LatentCholOracle(xv, y[perm], nb, 0, O.transform_latent(0, case["cov_pars"]), "poisson")
    assert abs(o.nll - case["nll"]) <= 1e-9 * abs(case["nll"]), (o.nll, case["nll"])
    np.testing.assert_allclose(o.grad()[0], case["grad"], rtol=1e-7)


def test_oracle_vif_mode_cap_matches_reference():
    case = GOLDEN["vif_pois_m40_nn15"]
    sp = case["spec"]
    X, y = _data(case["n"])
    perm, Z, _ = O.vif_inducing_points(X, sp["num_ind_points"], "kmeans++", 0, True)
    xv = X[perm]
    nb = O.find_neighbors(xv, sp["num_neighbors"])
    tr = O.transform_latent(0, case["cov_pars"])
    o = VifLaplaceOracle(xv, y[perm], nb, Z, 0, tr[0], tr[1], "poisson")
    assert abs(o.nll - case["nll"]) <= 1e-9 * abs(case["nll"]), (o.nll, case["nll"])
    np.testing.assert_allclose(o.grad()[0], case["grad"], rtol=1e-7)
