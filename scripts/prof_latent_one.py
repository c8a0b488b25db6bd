"""One warm-up and one profiled latent Vecchia nll+grad evaluation at n = 100k (for rocprofv3 kernel
traces and PMC passes). rocprofv3 --kernel-trace traces the default hipGraph replay path on this image
(profiles/r03/graph_replay_trace_result_r03.txt); GPBOOST_AMD_NO_GRAPH=1 launches the same kernels
eagerly, which the PMC scripts use so that every dispatch is attributed."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402

n = int(os.environ.get("N", "100000"))
lik = os.environ.get("LIK", "gaussian")
X = synthetic.bench_coords(n)
y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
gm = GPModel(gp_coords=X, likelihood=lik, cov_function="exponential",
             gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia", num_neighbors=30,
             matrix_inversion_method="iterative")
p = dict(num_rand_vec_trace=50)
if lik == "gaussian":
    p["init_aux_pars"] = [0.1]
gm.set_optim_params(p)
gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
t0 = time.time()
r = gm.neg_log_likelihood_and_grad([1.0, 0.1], None)
print(f"{lik} n={n} eval {time.time() - t0:.4f}s nll={r[0]:.10g} info={gm.last_iteration_info()}", flush=True)
