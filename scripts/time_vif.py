"""VIF (Gaussian, full-scale Vecchia) nll + grad at the bench leg's size (n = 100k, m = 200, nn = 30), 3 evaluations
(for kernel traces / PMC passes)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
X = synthetic.bench_coords(n)
Y = synthetic.bench_spatial_gaussian_y(X)
gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="full_scale_vecchia", num_ind_points=200,
             num_neighbors=30, seed=0)
gm.neg_log_likelihood_and_grad([0.1, 1.0, 0.1], Y, profile_sigma2=True)
for _ in range(3):
    t0 = time.perf_counter()
    r = gm.neg_log_likelihood_and_grad([0.1, 1.0, 0.1], None, profile_sigma2=True)
    print("vif s/eval", time.perf_counter() - t0, "nll", r[0], flush=True)
