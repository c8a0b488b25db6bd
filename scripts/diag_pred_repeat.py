"""Diagnostic (prints only): repeated latent predictions of one model."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gpboost_amd import GPModel, synthetic  # noqa: E402

case = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_latent_pred_1t.json")))["bern_obs_only_var"]
X = synthetic.bench_coords(case["n"])
y = synthetic.bench_bernoulli_y(X)
Xp = synthetic.lcg_unif(case["npred"] * 2, 0.713).reshape(2, case["npred"]).T.copy()
for draws in ("gpu", "reference"):
    os.environ["GPBOOST_AMD_PRED_DRAWS"] = draws
    for pv in (False, True):
        gm = GPModel(gp_coords=X, likelihood="bernoulli_logit", gp_approx="vecchia", num_neighbors=case["m"],
                     matrix_inversion_method="iterative", seed=0, cov_function="exponential")
        gm.set_optim_params(dict(num_rand_vec_trace=20, cg_delta_conv=1e-10))
        gm.set_prediction_data(vecchia_pred_type=case["ptype"], nsim_var_pred=case["nsim"])
        ref = np.asarray(case["mean"])
        for _ in range(3):
            r = gm.predict(y=y, gp_coords_pred=Xp, cov_pars=case["cov_pars"], predict_var=pv)
            print(draws, "var" if pv else "novar", float(np.max(np.abs(r["mu"] - ref))), gm.last_iteration_info(),
                  flush=True)
        nll = gm.neg_log_likelihood(case["cov_pars"], y)
        r2 = gm.predict(y=y, gp_coords_pred=Xp, cov_pars=case["cov_pars"], predict_var=pv)
        print("  after nll eval", float(np.max(np.abs(r2["mu"] - ref))), nll, flush=True)
