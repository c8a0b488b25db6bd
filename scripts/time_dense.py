"""Quick timing of the dense path at BASELINE config sizes (n=2000, n=20000)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from gpboost_amd import GPModel, synthetic
for n in [int(a) for a in sys.argv[1:]] or [2000, 20000]:
    X = synthetic.bench_coords(n); Y = synthetic.bench_gaussian_y(n)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="none")
    gm.neg_log_likelihood_and_grad([0.1, 1.0, 0.1], Y, profile_sigma2=True)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter(); r = gm.neg_log_likelihood_and_grad([0.1, 1.0, 0.1], None, profile_sigma2=True); ts.append(time.perf_counter() - t0)
    print(n, "s/eval", min(ts), "potrf_ms", gm.last_kernel_ms(), "nll", r[0], flush=True)
