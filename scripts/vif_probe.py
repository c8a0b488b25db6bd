"""VIF timing probe at the headline size (prints only): construction, nll + gradient per evaluation."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402

n = int(os.environ.get("VIF_N", "100000"))
m = int(os.environ.get("VIF_M", "200"))
nn = int(os.environ.get("VIF_NN", "30"))
X = synthetic.bench_coords(n)
y = synthetic.bench_spatial_gaussian_y(X)
t0 = time.perf_counter()
gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="full_scale_vecchia", num_ind_points=m, num_neighbors=nn)
print("construct_s", round(time.perf_counter() - t0, 3), flush=True)
th = [0.25, 1.0, 0.1]
r = gm.neg_log_likelihood_and_grad(th, y, profile_sigma2=True)
print("first", r[0], r[1], flush=True)
for want in (True, False):
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        if want:
            gm.neg_log_likelihood_and_grad(th, None, profile_sigma2=True)
        else:
            gm.neg_log_likelihood(th, y)
        ts.append(time.perf_counter() - t0)
    print("grad" if want else "nll_only", "ms", [round(1e3 * t, 2) for t in ts], "kernel_ms", gm.last_kernel_ms(), flush=True)
