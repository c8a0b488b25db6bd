"""Latent operator only, for PMC passes: one gaussian latent evaluation at n = 100k (factor),
then GPB_BenchLatentOperators at t = 1 (single-vector operator + preconditioner)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402

n = 100_000
X = synthetic.bench_coords(n)
y = synthetic.bench_gaussian_y(n)
gm = GPModel(gp_coords=X, likelihood="gaussian", cov_function="exponential", gp_approx="vecchia_latent",
             num_neighbors=30, vecchia_ordering="random", seed=0, matrix_inversion_method="iterative")
gm.set_optim_params(dict(num_rand_vec_trace=int(os.environ.get("T_PROBES", "4")), init_aux_pars=[0.1],
                         cg_delta_conv=1e-2))
gm.neg_log_likelihood([1.0, 0.1], y)
print(gm.bench_latent_operators(int(os.environ.get("T_OP", "1")), 20))
