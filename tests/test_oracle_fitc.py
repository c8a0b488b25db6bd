"""CPU: pin the FITC oracle (oracle/gp_oracle_fitc.cpp) to the reference itself
(tests/golden/golden_fitc.json, make_golden_fitc.py: oracle/_ref/ref_harness gp_approx=fitc).

The inducing points must be identical bit for bit (same std::mt19937 draws through
std::discrete_distribution / std::uniform_int_distribution, the reference's distance and mean
arithmetic in the Lloyd iterations); nll and gradient agree to 1e-9 relative (same formulas,
different summation order).
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import synthetic
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_fitc.json")) as _f:
    GOLDEN = json.load(_f)
SMALL = [k for k, v in GOLDEN.items() if "eval" in v and v["n"] <= 4000]


def _data(case):
    X = synthetic.bench_coords(case["n"])
    return X, synthetic.bench_spatial_gaussian_y(X)


@pytest.mark.parametrize("name", SMALL)
def test_inducing_points_bit_exact(name):
    case = GOLDEN[name]
    X, _ = _data(case)
    sp = case["spec"]
    Z, its = O.fitc_inducing_points(X, case["m"], sp["ind_points_selection"], int(sp["seed"]))
    ref = np.array(case["ind_points"]).reshape(case["m"], -1)
    assert np.array_equal(Z, ref), np.max(np.abs(Z - ref))


@pytest.mark.parametrize("name", SMALL)
@pytest.mark.parametrize("mode", [0, 1])
def test_nll_grad_matches_reference(name, mode):
    case = GOLDEN[name]
    X, y = _data(case)
    sp = case["spec"]
    ct = O.cov_code(sp["cov_fct"], float(sp["shape"]))
    Z = np.array(case["ind_points"]).reshape(case["m"], -1)
    r = O.fitc_nll_grad(X, y, Z, ct, O.transform(ct, case["cov_pars"]), mode)
    ref = case["eval" if mode == 0 else "lbfgs"]
    assert abs(r["nll"] - ref["nll"]) <= 1e-9 * abs(ref["nll"])
    np.testing.assert_allclose(r["grad"], ref["grad"], rtol=1e-8, atol=1e-9 * abs(ref["nll"]))
    assert abs(r["sigma2"] - ref["sigma2"]) <= 1e-10 * abs(ref["sigma2"])
