"""GPB_OptimCovPar for BASELINE config 5 (bernoulli_logit Laplace, Vecchia m=30, iterative, n=100k)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402

n = 100_000
X = synthetic.bench_coords(n)
y = synthetic.bench_bernoulli_y(X)
t0 = time.perf_counter()
gm = GPModel(gp_coords=X, likelihood="bernoulli_logit", cov_function="exponential", gp_approx="vecchia",
             num_neighbors=30, vecchia_ordering="random", seed=0, matrix_inversion_method="iterative")
gm.fit(y, params=dict(num_rand_vec_trace=50, cg_delta_conv=1e-2, seed_rand_vec_trace=1))
t = time.perf_counter() - t0
print(json.dumps({"s": t, "num_it": gm.get_num_optim_iter(), "nll": gm.get_current_neg_log_likelihood(),
                  "cov_pars": [float(v) for v in gm.get_cov_pars()], "init": [float(v) for v in gm.get_init_cov_pars()]}))
