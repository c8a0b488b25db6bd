"""Pins the order_pred_first restatement (oracle/pred_first_oracle.py) to the reference
(tests/golden/golden_pred_types.json): means elementwise at 1e-12, and the reference's variances /
covariance equal the restatement's under one permutation of the prediction points (the AMD ordering of
the reference's sparse Cholesky, Vecchia_utils.cpp:2220-2237), recovered from the variances and then
checked on the whole covariance matrix elementwise. CPU only."""
import json
import os

import numpy as np
import pytest

from gpboost_amd import synthetic
from oracle import oracle as O
from oracle.pred_first_oracle import pred_first

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_pred_types.json")) as _f:
    GOLDEN = json.load(_f)
NAMES = [k for k, v in GOLDEN.items() if v.get("ptype") == "order_pred_first"]


def run_case(case):
    sp = case["spec"]
    X = synthetic.bench_coords(case["n"])
    y = synthetic.bench_spatial_gaussian_y(X)
    npred = case["npred"]
    xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    ct = O.cov_code(sp["cov_fct"], float(sp["shape"]))
    return pred_first(X, y, xp, ct, O.transform(ct, case["cov_pars"]), int(sp["num_neighbors"]), case["mp"],
                      case["response"])


@pytest.mark.parametrize("name", NAMES)
def test_pred_first_oracle_matches_reference(name):
    case = GOLDEN[name]
    mean, cov = run_case(case)
    np.testing.assert_allclose(mean, case["mean"], rtol=1e-12, atol=1e-12)
    var = np.diag(cov)
    ref_c = np.asarray(case["cov"]).reshape(case["npred"], -1) if "cov" in case else None
    ref_v = np.diag(ref_c) if ref_c is not None else np.asarray(case["var"])
    # the permutation: the reference's k-th variance belongs to prediction point perm[k]
    assert len(np.unique(np.round(var, 12))) == len(var)   # distinct: the matching is unambiguous
    perm = np.argsort(var)[np.argsort(np.argsort(ref_v))]
    np.testing.assert_allclose(var[perm], ref_v, rtol=1e-12)
    assert sorted(perm.tolist()) == list(range(case["npred"]))
    if ref_c is not None:
        np.testing.assert_allclose(cov[np.ix_(perm, perm)], ref_c, rtol=1e-10, atol=1e-9 * np.abs(ref_c).max())
