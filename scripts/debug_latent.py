import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from gpboost_amd import GPModel, synthetic
from oracle import oracle as O

def run(n, m, t, lik, dc=1e-6, pars=(0.9, 0.2)):
    X = synthetic.bench_coords(n)
    y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
    gm = GPModel(gp_coords=X, likelihood=lik, gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia",
                 cov_function="exponential", num_neighbors=m, matrix_inversion_method="iterative")
    p = dict(num_rand_vec_trace=t, seed_rand_vec_trace=2, cg_delta_conv=dc)
    if lik == "gaussian":
        p["init_aux_pars"] = [0.4]
    gm.set_optim_params(p)
    nll, g, _ = gm.neg_log_likelihood_and_grad(list(pars), y)
    mm = min(m, n - 1)
    perm, xv, nb = O.vecchia_setup(X, mm, 0, True)
    ref = O.latent_iterative(xv, y[perm], nb, 0, O.transform_latent(0, list(pars)), lik, 0.4, t=t, seed=2, cg_delta_conv=dc)
    print(n, m, t, lik, dc, "gpu", nll, g, gm.last_iteration_info(), "| orc", ref["nll"], ref["grad"],
          ref["newton_its"], ref["cg_its"], ref["lanczos_steps"], ref["logdet"], flush=True)

for args in [(400, 1, 1, "bernoulli_logit"), (400, 1, 2, "bernoulli_logit"), (400, 8, 1, "bernoulli_logit"),
             (400, 8, 4, "bernoulli_logit"), (400, 1, 1, "gaussian"), (400, 8, 1, "gaussian"),
             (5, 3, 7, "gaussian"), (600, 8, 70, "gaussian"), (50, 49, 4, "bernoulli_logit")]:
    run(*args)
run(20000, 30, 10, "bernoulli_logit", 1e-8, (1.0, 0.1))
run(20000, 30, 10, "gaussian", 1e-8, (1.0, 0.1))
