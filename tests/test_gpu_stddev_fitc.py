"""GPU parity for the standard deviations of the covariance parameters of the Gaussian FITC model
(GPB_GetCovPar(calc_std_dev = true) -> CalcStdDevCovPar re_model_template.h:9775-9789 ->
CalcFisherInformation_FITC_FSA :9363-9548, cholesky) through the C ABI.

Fixtures: tests/golden/golden_stddev_fitc.json (the reference itself, make_golden_stddev_fitc.py), to which
the CPU restatement (oracle/fitc_fisher_oracle.py) is pinned at 1e-9 by test_oracle_stddev_fitc.py. Same
probes as the reference, so only rounding separates the estimates: 1e-8 relative.
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPModel, synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_stddev_fitc.json")) as _f:
    GOLDEN = json.load(_f)


def _model(c):
    sp = c["spec"]
    X = synthetic.bench_coords(c["n"])
    gm = GPModel(gp_coords=X, cov_function=sp["cov_fct"], cov_fct_shape=float(sp["shape"]), gp_approx="fitc",
                 num_ind_points=int(sp["num_ind_points"]), ind_points_selection=sp["ind_points_selection"],
                 seed=int(sp["seed"]))
    p = {}
    if c["num_rand_vec_trace"] is not None:
        p["num_rand_vec_trace"] = c["num_rand_vec_trace"]
    if c["seed_rand_vec_trace"] is not None:
        p["seed_rand_vec_trace"] = c["seed_rand_vec_trace"]
    if p:
        gm.set_optim_params(p)
    return gm, X, synthetic.bench_spatial_gaussian_y(X)


@pytest.mark.parametrize("name", list(GOLDEN))
def test_stddev_fitc_matches_reference(name):
    c = GOLDEN[name]
    gm, X, y = _model(c)
    assert gm.can_calculate_standard_errors_cov_pars()
    gm.neg_log_likelihood(c["cov_pars"], y)
    out = gm.get_cov_pars(std_err=True)
    np.testing.assert_allclose(out[0], c["cov_pars"], rtol=1e-15)
    np.testing.assert_allclose(out[1], c["std_dev"], rtol=1e-8)


def test_stddev_fitc_after_fit_vs_oracle():
    """After a fit: the standard deviations at the estimates, against the oracle (m = 7: one MFMA tile with
    padding; t = 5 probes)."""
    from oracle import oracle as O
    from oracle.fitc_fisher_oracle import fitc_fisher
    n, m = 800, 7
    X = synthetic.bench_coords(n)
    y = synthetic.bench_spatial_gaussian_y(X)
    gm = GPModel(gp_coords=X, cov_function="matern", cov_fct_shape=1.5, gp_approx="fitc", num_ind_points=m, seed=2)
    gm.fit(y, params={"num_rand_vec_trace": 5, "seed_rand_vec_trace": 11})
    est = gm.get_cov_pars(std_err=True)
    Z, _ = O.fitc_inducing_points(X, m, "kmeans++", 2)
    _, ref = fitc_fisher(X, Z, 1, est[0], t=5, seed=11)
    np.testing.assert_allclose(est[1], ref, rtol=1e-8)
