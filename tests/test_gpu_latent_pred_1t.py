"""Laplace predictive variances and covariances (Vecchia, iterative) against the reference's OWN draws:
tests/golden/golden_latent_pred_1t.json is the reference run on one thread (make_golden_latent_pred_1t.py),
whose simulation (PredictLaplaceApproxVecchia, likelihoods.h:6668-6700) draws one mt19937 stream seeded from
the likelihood's default-seeded cg_generator_. With GPBOOST_AMD_PRED_DRAWS=reference gpboost_amd draws the
same stream on the host, so the simulated moments match elementwise to the CG tolerance (cg_delta_conv =
1e-10): mean and variances / covariances 1e-6 relative (north-star tolerance), in place of the
statistical bound of test_gpu_latent_pred.py.
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPModel, synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_latent_pred_1t.json")) as _f:
    GOLDEN = json.load(_f)


@pytest.mark.parametrize("name", list(GOLDEN))
def test_latent_pred_reference_draws(monkeypatch, name):
    monkeypatch.setenv("GPBOOST_AMD_PRED_DRAWS", "reference")
    case = GOLDEN[name]
    n, npred = case["n"], case["npred"]
    X = synthetic.bench_coords(n)
    y = synthetic.bench_poisson_y(X) if case["lik"] == "poisson" else synthetic.bench_bernoulli_y(X)
    Xp = synthetic.lcg_unif(npred * 2, 0.713).reshape(2, npred).T.copy()
    gm = GPModel(gp_coords=X, likelihood=case["lik"], cov_function="exponential", gp_approx="vecchia",
                 num_neighbors=case["m"], vecchia_ordering="random", matrix_inversion_method="iterative", seed=0)
    gm.set_optim_params(dict(num_rand_vec_trace=20, cg_delta_conv=1e-10))
    gm.set_prediction_data(vecchia_pred_type=case["ptype"], nsim_var_pred=case["nsim"])
    want_cov = "cov" in case
    pred = gm.predict(y=y, gp_coords_pred=Xp, cov_pars=case["cov_pars"], predict_var=not want_cov,
                      predict_cov_mat=want_cov, predict_response=case["response"])
    # the mode to the CG tolerance; cond_all's mean (-Bp^-1 Bpo mode) carries its conditioning
    np.testing.assert_allclose(pred["mu"], case["mean"], rtol=1e-6, atol=1e-10)
    if want_cov:
        ref = np.asarray(case["cov"]).reshape(npred, npred)
        np.testing.assert_allclose(pred["cov"], ref, rtol=1e-6, atol=1e-6 * np.abs(ref).max())
    else:
        np.testing.assert_allclose(pred["var"], case["var"], rtol=1e-6, atol=1e-10)


def test_reference_draws_continue_the_generator(monkeypatch):
    """A second prediction of the same model continues the likelihood's generator (a new stream seed), so
    its simulated variances differ from the first call's; the deterministic part (the means) does not."""
    monkeypatch.setenv("GPBOOST_AMD_PRED_DRAWS", "reference")
    case = GOLDEN["bern_obs_only_var"]
    X = synthetic.bench_coords(case["n"])
    y = synthetic.bench_bernoulli_y(X)
    Xp = synthetic.lcg_unif(case["npred"] * 2, 0.713).reshape(2, case["npred"]).T.copy()
    gm = GPModel(gp_coords=X, likelihood="bernoulli_logit", cov_function="exponential", gp_approx="vecchia",
                 num_neighbors=case["m"], vecchia_ordering="random", matrix_inversion_method="iterative", seed=0)
    gm.set_optim_params(dict(num_rand_vec_trace=20, cg_delta_conv=1e-10))
    gm.set_prediction_data(vecchia_pred_type=case["ptype"], nsim_var_pred=case["nsim"])
    a = gm.predict(y=y, gp_coords_pred=Xp, cov_pars=case["cov_pars"], predict_var=True, predict_response=False)
    b = gm.predict(y=y, gp_coords_pred=Xp, cov_pars=case["cov_pars"], predict_var=True, predict_response=False)
    np.testing.assert_array_equal(a["mu"], b["mu"])
    assert not np.allclose(a["var"], b["var"], rtol=1e-9)
    np.testing.assert_allclose(a["var"], case["var"], rtol=1e-6, atol=1e-10)
