"""GPU parity for the standard deviations of the covariance parameters of the Gaussian Vecchia model
(GPB_GetCovPar(calc_std_dev = true) -> CalcStdDevCovPar re_model_template.h:9775-9789 ->
CalcFisherInformation_Vecchia :9246-9298, the reference's default stochastic-trace form) through the C ABI.

Fixtures: tests/golden/golden_stddev_vecchia.json (the reference itself, make_golden_stddev_vecchia.py), to
which the CPU restatement (oracle/vecchia_fisher_oracle.py) is pinned at 1e-12 by
test_oracle_stddev_vecchia.py. The probes are the reference's own (GenRandVecNormalParallel), so only
rounding separates the GPU estimate from the reference's: 1e-8 relative (fp64 throughout; the VADU head
solves through an explicit inverse of the first 2048 rows, hence not 1e-12).
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPBoostError, GPModel, synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_stddev_vecchia.json")) as _f:
    GOLDEN = json.load(_f)


def _model(c):
    sp = c["spec"]
    X = synthetic.bench_coords(c["n"])
    gm = GPModel(gp_coords=X, cov_function=sp["cov_fct"], cov_fct_shape=float(sp["shape"]), gp_approx="vecchia",
                 num_neighbors=int(sp["num_neighbors"]), vecchia_ordering=sp["ordering"], seed=int(sp["seed"]))
    p = {}
    if c["num_rand_vec_trace"] is not None:
        p["num_rand_vec_trace"] = c["num_rand_vec_trace"]
    if c["seed_rand_vec_trace"] is not None:
        p["seed_rand_vec_trace"] = c["seed_rand_vec_trace"]
    if p:
        gm.set_optim_params(p)
    return gm, X, synthetic.bench_spatial_gaussian_y(X)


@pytest.mark.parametrize("name", list(GOLDEN))
def test_stddev_vecchia_matches_reference(name):
    c = GOLDEN[name]
    gm, X, y = _model(c)
    assert gm.can_calculate_standard_errors_cov_pars()
    gm.neg_log_likelihood(c["cov_pars"], y)   # sets the parameters GPB_GetCovPar reports
    out = gm.get_cov_pars(std_err=True)
    np.testing.assert_allclose(out[0], c["cov_pars"], rtol=1e-15)
    np.testing.assert_allclose(out[1], c["std_dev"], rtol=1e-8)


def test_stddev_vecchia_vs_oracle_small_and_head_splits(monkeypatch):
    """Tiny n (rows with fewer than num_neighbors neighbours dominate), and the same model with the VADU
    plan's dense head / LDS segment switched off (GPBOOST_AMD_DENSE_ROWS / HEAD_ROWS = 0: every row in the
    level-scheduled tail): the same estimate as the oracle either way."""
    from oracle import oracle as O
    from oracle.vecchia_fisher_oracle import vecchia_fisher
    cp = [0.2, 1.1, 0.12]
    for n, nn, env in [(40, 12, None), (1200, 10, None), (1200, 10, "0")]:
        if env is not None:
            monkeypatch.setenv("GPBOOST_AMD_DENSE_ROWS", env)
            monkeypatch.setenv("GPBOOST_AMD_HEAD_ROWS", env)
        X = synthetic.bench_coords(n)
        y = synthetic.bench_spatial_gaussian_y(X)
        gm = GPModel(gp_coords=X, cov_function="matern", cov_fct_shape=1.5, gp_approx="vecchia", num_neighbors=nn,
                     seed=5)
        gm.set_optim_params({"num_rand_vec_trace": 16, "seed_rand_vec_trace": 3})
        gm.neg_log_likelihood(cp, y)
        sd = gm.get_cov_pars(std_err=True)[1]
        _, xv, nb = O.vecchia_setup(X, min(nn, n - 1), 5, True)
        _, ref = vecchia_fisher(xv, nb, 1, cp, t=16, seed=3)
        np.testing.assert_allclose(sd, ref, rtol=1e-8, err_msg=f"n={n} env={env}")


def test_stddev_vecchia_after_fit():
    """After a fit the standard deviations are those at the estimates (re_model.cpp:785-810)."""
    c = GOLDEN["sdv_exp_n1000_nn8_none"]
    gm, X, y = _model(c)
    gm.fit(y)
    est = gm.get_cov_pars(std_err=True)
    assert np.all(np.isfinite(est[1])) and np.all(est[1] > 0)
    from oracle import oracle as O
    from oracle.vecchia_fisher_oracle import vecchia_fisher
    _, xv, nb = O.vecchia_setup(X, 8, 0, False)
    _, ref = vecchia_fisher(xv, nb, 0, est[0], t=50, seed=1)
    np.testing.assert_allclose(est[1], ref, rtol=1e-8)


def test_stddev_refusals():
    X = synthetic.bench_coords(300)
    y = synthetic.bench_spatial_gaussian_y(X)
    gl = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=10,
                 likelihood="bernoulli_logit")
    assert not gl.can_calculate_standard_errors_cov_pars()
    gv = GPModel(gp_coords=X, gp_approx="vif", num_ind_points=20, num_neighbors=10, cov_function="exponential")
    assert not gv.can_calculate_standard_errors_cov_pars()   # re_model_template.h:1649-1651
    gv.neg_log_likelihood([0.1, 1.0, 0.1], y)
    with pytest.raises(GPBoostError, match="standard deviations"):
        gv.get_cov_pars(std_err=True)
