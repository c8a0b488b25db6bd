"""Time the latent Vecchia iterative evaluation (nll + grad) at BASELINE sizes on the GPU."""
import sys
import time

import numpy as np

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402


def run(lik, n, reps=3, t=50):
    X = synthetic.bench_coords(n)
    y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
    gm = GPModel(gp_coords=X, likelihood=lik, cov_function="exponential",
                 gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia", num_neighbors=30,
                 matrix_inversion_method="iterative")
    p = dict(num_rand_vec_trace=t)
    if lik == "gaussian":
        p["init_aux_pars"] = [0.1]
    gm.set_optim_params(p)
    t0 = time.time()
    r = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
    print(f"{lik} n={n} first eval {time.time() - t0:.3f}s nll={r[0]:.10g} grad={r[1]}", flush=True)
    ts = []
    for _ in range(reps):
        t0 = time.time()
        gm.neg_log_likelihood_and_grad([1.0, 0.1], None)
        ts.append(time.time() - t0)
    info = gm.last_iteration_info()
    print(f"{lik} n={n} eval {np.median(ts):.4f}s (device {gm.last_kernel_ms()[1]:.2f} ms) info={info}", flush=True)


if __name__ == "__main__":
    for lik in sys.argv[1:] or ["gaussian", "bernoulli_logit"]:
        for n in [int(v) for v in os.environ.get("SIZES", "20000 100000").split()]:
            run(lik, n)
