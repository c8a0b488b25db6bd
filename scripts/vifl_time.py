"""Timing probe: VIF Laplace (bernoulli_logit, cholesky) nll + grad at n = 20k / 100k, m = 200, nn = 30."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPBOOST_AMD_TIMING", "1")
from gpboost_amd import GPModel, synthetic  # noqa: E402

for n in [int(a) for a in sys.argv[1:]] or [20000, 100000]:
    X = synthetic.bench_coords(n)
    y = synthetic.bench_bernoulli_y(X)
    t0 = time.perf_counter()
    gm = GPModel(gp_coords=X, likelihood="bernoulli_logit", cov_function="exponential", gp_approx="full_scale_vecchia",
                 num_ind_points=200, num_neighbors=30, seed=0, matrix_inversion_method="cholesky")
    r = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
    t1 = time.perf_counter()
    ts = []
    for _ in range(3):
        a = time.perf_counter()
        r = gm.neg_log_likelihood_and_grad([1.0, 0.1], None)
        ts.append(time.perf_counter() - a)
    a = time.perf_counter()
    nll = gm.neg_log_likelihood([1.0, 0.1], None)
    tn = time.perf_counter() - a
    print(f"n={n}: first {t1 - t0:.2f} s, nll+grad {np.median(ts) * 1e3:.1f} ms, nll only {tn * 1e3:.1f} ms, "
          f"nll {r[0]:.10f} grad {r[1]}, plan {gm.cholesky_plan_info() if hasattr(gm, 'cholesky_plan_info') else None}",
          flush=True)
