"""GPU parity for predictions with the full-scale Vecchia approximation ("VIF", gp_approx = "full_scale_vecchia",
Gaussian likelihood): CalcPredVecchiaObservedFirstOrder's full-scale branches
(Vecchia_utils.cpp:1686-1707, 1826-1840, 1872-1873, 1901-1980; re_model_template.h:3708-3792) through the C ABI
(csrc/vif_kernels.hip VifSolver::Predict).

Fixtures: tests/golden/golden_vif_pred.json (the reference itself, make_golden_vif_pred.py): means with variances
or covariance matrices, latent and response, order_obs_first_cond_obs_only and order_obs_first_cond_all, three
covariance functions. Both sides are exact algebra on the same approximation: 1e-8 relative.
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import GPBoostError, GPModel, synthetic

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_vif_pred.json")) as _f:
    GOLDEN = json.load(_f)


@pytest.mark.parametrize("name", list(GOLDEN))
def test_vif_predict_matches_reference(name):
    c = GOLDEN[name]
    sp = c["spec"]
    X = synthetic.bench_coords(c["n"])
    y = synthetic.bench_spatial_gaussian_y(X)
    xp = synthetic.lcg_unif(c["npred"] * 2, 0.713).reshape(2, c["npred"]).T.copy()
    if c["dup5"]:
        xp[:5] = X[:5]
    gm = GPModel(gp_coords=X, cov_function=sp["cov_fct"], cov_fct_shape=float(sp["shape"]), gp_approx="full_scale_vecchia",
                 num_ind_points=int(sp["num_ind_points"]), num_neighbors=int(sp["num_neighbors"]),
                 vecchia_ordering=sp["ordering"], ind_points_selection=sp["ind_points_selection"], seed=int(sp["seed"]))
    kw = dict(vecchia_pred_type=c["vecchia_pred_type"])
    if c["num_neighbors_pred"] > 0:
        kw["num_neighbors_pred"] = c["num_neighbors_pred"]
    gm.set_prediction_data(**kw)
    want_cov = "cov" in c
    pred = gm.predict(y=y, gp_coords_pred=xp, cov_pars=c["cov_pars"], predict_var=not want_cov,
                      predict_cov_mat=want_cov, predict_response=c["response"])
    mu = np.asarray(c["mean"])
    np.testing.assert_allclose(pred["mu"], mu, rtol=1e-8, atol=1e-9 * np.abs(mu).max())
    if want_cov:
        cov = np.asarray(c["cov"]).reshape(c["npred"], c["npred"])
        np.testing.assert_allclose(pred["cov"], cov, rtol=1e-8, atol=1e-9 * np.abs(cov).max())
    else:
        np.testing.assert_allclose(pred["var"], c["var"], rtol=1e-8, atol=1e-11)


def test_vif_predict_refusals():
    X = synthetic.bench_coords(300)
    y = synthetic.bench_spatial_gaussian_y(X)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="full_scale_vecchia", num_ind_points=20,
                 num_neighbors=5)
    gm.set_prediction_data(vecchia_pred_type="order_pred_first")
    with pytest.raises(GPBoostError, match="prediction locations appear first"):
        gm.predict(y=y, gp_coords_pred=X[:4] + 0.01, cov_pars=[0.1, 1.0, 0.1], predict_var=True)
