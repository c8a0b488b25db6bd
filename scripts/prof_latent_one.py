"""One latent evaluation (for rocprofv3 kernel traces)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402

lik = sys.argv[1] if len(sys.argv) > 1 else "gaussian"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
X = synthetic.bench_coords(n)
y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
gm = GPModel(gp_coords=X, likelihood=lik, cov_function="exponential",
             gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia", num_neighbors=30,
             matrix_inversion_method="iterative")
p = dict(num_rand_vec_trace=50)
if len(sys.argv) > 3:   # cap the CG iterations (short profiles)
    p.update(cg_max_num_it=int(sys.argv[3]), cg_max_num_it_tridiag=int(sys.argv[3]))
if lik == "gaussian":
    p["init_aux_pars"] = [0.1]
gm.set_optim_params(p)
r = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
print(r, gm.last_iteration_info(), gm.last_kernel_ms())
