"""Diagnostic: FITC-Laplace on the GPU against the numpy oracle over likelihoods / kernels (prints only)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lik_case_data  # noqa: E402
from gpboost_amd import GPModel, synthetic  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle.fitc_laplace_oracle import FitcLaplaceOracle  # noqa: E402

G = json.load(open(os.path.join(ROOT, "tests", "golden", "golden_latent_lik.json")))
base = G["fp_pois_gauss_n2500_m60_random"]
for lik, cov, shape, cp, sel in [("poisson", "gaussian", 0.0, (0.6, 0.2), "random"),
                                 ("poisson", "gaussian", 0.0, (0.6, 0.05), "random"),
                                 ("poisson", "exponential", 0.5, (0.6, 0.2), "random"),
                                 ("bernoulli_logit", "gaussian", 0.0, (0.6, 0.2), "random"),
                                 ("bernoulli_probit", "gaussian", 0.0, (0.6, 0.2), "random"),
                                 ("poisson", "gaussian", 0.0, (0.6, 0.2), "kmeans++")]:
    case = dict(base, likelihood=lik, data="bench_pois" if lik == "poisson" else "bench_bern")
    X, y = lik_case_data(case)
    gm = GPModel(gp_coords=X, cov_function=cov, cov_fct_shape=shape, gp_approx="fitc", num_ind_points=60,
                 likelihood=lik, ind_points_selection=sel, seed=3)
    nll, g, _ = gm.neg_log_likelihood_and_grad(list(cp), y)
    Z = O.fitc_inducing_points(X, 60, sel, 3)[0]
    ct = O.cov_code(cov, shape)
    tr = O.transform_latent(ct, list(cp))
    o = FitcLaplaceOracle(X, y, Z, ct, tr[0], tr[1], likelihood=lik)
    onll = o.find_mode()
    og = o.gradient()["grad"]
    print(lik, cov, cp, sel, "gpu", repr(nll), "oracle", repr(onll), "its", o.newton_its, "rel", (nll - onll) / onll,
          "grad", g, og, "cond", np.linalg.cond(o.Ks), flush=True)
    print("  info", gm.last_iteration_info(), flush=True)
