"""Rounding sensitivity of the latent (PCG + SLQ) evaluation at n = 100k, default tolerance: the same
evaluation under algebraically equivalent preconditioner plans / storage orders (env settings from
the command line, one per process). Prints nll, gradient and [newton its, CG its, Lanczos steps, logdet]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402

n = int(os.environ.get("N", "100000"))
X = synthetic.bench_coords(n)
lik = os.environ.get("LIK", "gaussian")
y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
gm = GPModel(gp_coords=X, likelihood=lik, cov_function="exponential",
             gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia",
             num_neighbors=30, vecchia_ordering="random", seed=0, matrix_inversion_method="iterative")
p = dict(num_rand_vec_trace=50, cg_delta_conv=float(os.environ.get("DC", "1e-2")), seed_rand_vec_trace=1)
if lik == "gaussian":
    p["init_aux_pars"] = [0.1]
gm.set_optim_params(p)
nll, g, _ = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
print(os.environ.get("TAG", "default"), repr(nll), [float(v) for v in g], list(gm.last_iteration_info()), flush=True)
