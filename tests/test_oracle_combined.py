"""The dense CPU restatement of the combined GP + grouped random effects likelihood
(oracle/combined_oracle.py) pinned to the reference's own outputs (tests/golden/golden_combined.json,
make_golden_combined.py from oracle/_ref/ref_harness with group labels): nll 1e-10, gradient 1e-8."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from oracle.combined_oracle import combined_nll_grad

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_combined.json")) as _f:
    GOLDEN = json.load(_f)

import sys  # noqa: E402
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_golden_combined import data  # noqa: E402


@pytest.mark.parametrize("name", [k for k in GOLDEN if k.startswith("cb_")])
def test_oracle_combined_matches_reference(name):
    c = GOLDEN[name]
    X, g, y = data(c["kind"], c["n"], tuple(c["levels"]))
    sp = c["spec"]
    ct = O.cov_code(sp["cov_fct"], float(sp["shape"]))
    cp = np.array(c["cov_pars"], float)
    K = g.shape[1]
    trafo = np.concatenate([[cp[0]], cp[1:1 + K] / cp[0], [cp[1 + K] / cp[0]],
                            [O.transform(ct, [cp[0], cp[1 + K], cp[2 + K]])[2]]])
    r = combined_nll_grad(X, g, y, ct, trafo, mode=0)
    assert abs(r["nll"] - c["nll"]) <= 1e-10 * abs(c["nll"])
    np.testing.assert_allclose(r["grad"], c["grad"], rtol=1e-8, atol=1e-10 * abs(c["nll"]))
    p = combined_nll_grad(X, g, y, ct, trafo, mode=1)
    assert abs(p["nll"] - c["lbfgs_nll"]) <= 1e-10 * abs(c["lbfgs_nll"])
    np.testing.assert_allclose(p["grad"], c["lbfgs_grad"], rtol=1e-8, atol=1e-10 * abs(c["nll"]))
