"""Per-evaluation host overhead of the exact path: wall time per nll+grad evaluation vs the row
kernel's HIP-event time, and the bare C-ABI call without the Python mirror's argument checks."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402

n = 100_000
X = synthetic.bench_coords(n)
Y = synthetic.bench_gaussian_y(n)
gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=30, vecchia_ordering="random",
             seed=0)
th = [0.1, 1.0, 0.1]
gm.neg_log_likelihood_and_grad(th, Y, profile_sigma2=True)
for _ in range(20):
    gm.neg_log_likelihood_and_grad(th, None, profile_sigma2=True)
reps = 500
t0 = time.perf_counter()
for _ in range(reps):
    gm.neg_log_likelihood_and_grad(th, None, profile_sigma2=True)
wall = (time.perf_counter() - t0) / reps * 1e3
gm.last_kernel_ms()   # switch event recording on
ks = []
for _ in range(20):
    gm.neg_log_likelihood_and_grad(th, None, profile_sigma2=True)
    ks.append(gm.last_kernel_ms())
ks = np.array(ks)
print(f"wall {wall:.4f} ms/eval, row kernel {ks[:, 0].mean():.4f} ms, kernel+sum {ks[:, 1].mean():.4f} ms, "
      f"evals/s {1e3 / wall:.1f}")

# the bare C-ABI call (pre-built ctypes pointers, no argument checks)
import ctypes  # noqa: E402
from gpboost_amd.basic import _dp, lib  # noqa: E402
L = lib()
cp = np.array(th)
negll, grad, s2 = np.zeros(1), np.zeros(3), np.zeros(1)
pc, pn, pg, ps = _dp(cp), _dp(negll), _dp(grad), _dp(s2)
f = L.GPB_EvalNegLogLikelihoodGrad
for _ in range(20):
    f(gm.handle, None, pc, None, 1, pn, pg, ps)
t0 = time.perf_counter()
for _ in range(reps):
    f(gm.handle, None, pc, None, 1, pn, pg, ps)
bare = (time.perf_counter() - t0) / reps * 1e3
print(f"bare C call {bare:.4f} ms/eval")

# one-rank RCCL communicator: the N > 1 code path (sum kernel to device, ncclAllReduce, D2H copy)
from gpboost_amd import comm_create_id  # noqa: E402
g2 = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=30, vecchia_ordering="random",
             seed=0)
g2.set_distributed(0, 1, comm_create_id())
g2.neg_log_likelihood_and_grad(th, Y, profile_sigma2=True)
for _ in range(20):
    f(g2.handle, None, pc, None, 1, pn, pg, ps)
t0 = time.perf_counter()
for _ in range(reps):
    f(g2.handle, None, pc, None, 1, pn, pg, ps)
rc = (time.perf_counter() - t0) / reps * 1e3
print(f"bare C call through a one-rank RCCL communicator {rc:.4f} ms/eval (+{(rc - bare) * 1e3:.1f} us)")
