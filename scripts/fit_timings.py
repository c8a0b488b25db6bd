"""GPB_OptimCovPar wall times on the BASELINE configurations beyond the headline (GPU only):
vecchia_latent gaussian (config 3b) at n=100k and the dense GP (config 2) at n=20000."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402

out = {}
n = 100_000
X = synthetic.bench_coords(n)
y = synthetic.bench_gaussian_y(n)
t0 = time.perf_counter()
gm = GPModel(gp_coords=X, likelihood="gaussian", cov_function="exponential", gp_approx="vecchia_latent",
             num_neighbors=30, vecchia_ordering="random", seed=0, matrix_inversion_method="iterative")
gm.fit(y, params=dict(num_rand_vec_trace=50, cg_delta_conv=1e-2))
out["vecchia_latent_100k"] = {"s": time.perf_counter() - t0, "num_it": gm.get_num_optim_iter(),
                              "nll": gm.get_current_neg_log_likelihood(),
                              "cov_pars": [float(v) for v in gm.get_cov_pars()],
                              "aux": [float(v) for v in gm.get_aux_pars()[0]]}
print(json.dumps(out), flush=True)
del gm
n = 20_000
X = synthetic.bench_coords(n)
y = synthetic.bench_gaussian_y(n)
t0 = time.perf_counter()
gm = GPModel(gp_coords=X, cov_function="exponential")
gm.fit(y)
out["dense_20k"] = {"s": time.perf_counter() - t0, "num_it": gm.get_num_optim_iter(),
                    "nll": gm.get_current_neg_log_likelihood(), "cov_pars": [float(v) for v in gm.get_cov_pars()]}
t0 = time.perf_counter()
sd = gm.get_cov_pars(std_err=True)[1]
out["dense_20k"]["std_err_s"] = time.perf_counter() - t0
out["dense_20k"]["std_err"] = [float(v) for v in sd]
print(json.dumps(out), flush=True)
