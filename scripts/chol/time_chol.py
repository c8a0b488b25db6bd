"""Timing of the latent Vecchia Cholesky path (matrix_inversion_method = "cholesky") at BASELINE sizes.
    python scripts/chol/time_chol.py 100000 [reps]
Prints per-evaluation wall times of nll + gradient; GPBOOST_AMD_TIMING=1 adds the device-side breakdown."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from gpboost_amd import GPModel, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
lik = sys.argv[3] if len(sys.argv) > 3 else "bernoulli_logit"
X = synthetic.bench_coords(n)
y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
t0 = time.time()
gm = GPModel(gp_coords=X, likelihood=lik, cov_function="exponential", gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia",
             num_neighbors=30, vecchia_ordering="random", matrix_inversion_method="cholesky", seed=0)
if lik == "gaussian":
    gm.set_optim_params(dict(init_aux_pars=[0.1], estimate_aux_pars=True))
nll = gm.neg_log_likelihood([1.0, 0.1], y)
t1 = time.time()
print(f"n={n} construction + first nll {t1 - t0:.2f} s nll={nll!r}", flush=True)
for r in range(reps):
    a = time.time()
    nll, g, _ = gm.neg_log_likelihood_and_grad([1.0, 0.1], y if r == 0 else None)
    b = time.time()
    print(f"  eval {r}: {1e3 * (b - a):.1f} ms nll={nll!r} grad={g}", flush=True)
