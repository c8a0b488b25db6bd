"""GPU parity of the Newton mode-change cap for count likelihoods (CapChangeModeUpdateNewton, likelihoods.h:11800-11810;
poisson / gamma in the Vecchia and full-scale Vecchia mode finding, :2974, :2606) against the reference's own values
for Poisson counts of a few hundred (tests/golden/golden_mode_cap.json): the first Newton step from mode 0 exceeds
log(100) and is capped. nll 1e-9, gradient 1e-7 (exact Cholesky paths)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_mode_cap.json")) as _f:
    GOLDEN = json.load(_f)


@pytest.mark.parametrize("name", list(GOLDEN))
def test_mode_cap_matches_reference(name):
    from gpboost_amd import GPModel, synthetic
    case = GOLDEN[name]
    sp = case["spec"]
    X = synthetic.bench_coords(case["n"])
    y = np.round(300. * np.exp(np.sin(4. * X[:, 0]) * np.cos(3. * X[:, 1])))
    kw = dict(num_neighbors=sp["num_neighbors"], matrix_inversion_method="cholesky", seed=0)
    if sp["gp_approx"] == "full_scale_vecchia":
        kw["num_ind_points"] = sp["num_ind_points"]
    else:
        kw["vecchia_ordering"] = "random"
    gm = GPModel(gp_coords=X, likelihood="poisson", cov_function="exponential", gp_approx=sp["gp_approx"], **kw)
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= 1e-9 * abs(case["nll"]), (nll, case["nll"])
    np.testing.assert_allclose(g, case["grad"], rtol=1e-7)
