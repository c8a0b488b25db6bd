"""Pins the internal-optimizer restatement (oracle/internal_optim_oracle.py: the reference's gradient
descent with Nesterov momentum and Fisher scoring, re_model_template.h:1290-1549) to the reference: the
fits of tests/golden/golden_internal_optim.json (make_golden_internal_optim.py) on the R tests' data are
reproduced with identical iteration counts and estimates to 1e-7 relative (the restatement's dense
numpy algebra differs from the reference's Eigen Cholesky only in rounding)."""
import json
import os

import numpy as np
import pytest

from gpboost_amd import synthetic
from oracle.internal_optim_oracle import DenseModel, internal_optimize

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(HERE, "golden", "golden_internal_optim.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["rtest_gd_nesterov", "rtest_gd_no_acc", "rtest_gd_lr1", "rtest_gd_crit_pars",
                                  "rtest_fisher", "combined_rtest_gd"])
def test_internal_optim_oracle_matches_reference(golden, name):
    case = golden[name]
    sp = case["spec"]
    if case["data"] == "rtest_combined":
        X, g, y = synthetic.rtest_combined_y(100)
    else:
        (X, y), g = synthetic.rtest_gaussian_y(100), None
    m = DenseModel(X, g, y, cov_type=0)   # exponential: phi = 1 / rho
    init = np.array(case["init_cov_pars"], float)
    s2 = init[0]
    trafo = np.concatenate([[s2], init[1:-1] / s2, [1. / init[-1]]])
    pars, nll, num_it = internal_optimize(
        m, trafo, sp["optimizer"], lr=float(sp.get("lr_cov", -1)), nesterov=sp.get("use_nesterov_acc", "1") != "0",
        delta=float(sp.get("delta_rel_conv", 1e-6)),
        crit_params=sp.get("convergence_criterion") == "relative_change_in_parameters")
    est = np.concatenate([[pars[0]], pars[1:-1] * pars[0], [1. / pars[-1]]])
    assert num_it == case["num_it"]
    np.testing.assert_allclose(est, case["cov_pars"], rtol=1e-7)
    assert abs(nll - case["nll"]) <= 1e-10 * abs(case["nll"])
