"""Exact-path row-shard wall time probe (e1): the per-rank row range of an N-rank run evaluated on one GPU,
timed with and without the kernel HIP events, at the bench's headline data (n = 100k, m = 30)."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from gpboost_amd import GPModel, synthetic  # noqa: E402

N, M = 100_000, 30
THETA = [0.1, 1.0, 0.1]
X = synthetic.bench_coords(N)
Y = synthetic.bench_gaussian_y(N)
gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=M,
             vecchia_ordering="random", seed=0)
gm.neg_log_likelihood_and_grad(THETA, Y, profile_sigma2=True)
t_end = time.perf_counter() + 0.5
while time.perf_counter() < t_end:   # clock ramp
    gm.vecchia_partials(THETA, 0, N)

out = {}
reps = 400
for nr in (1, 2, 4, 8):
    base = N // nr
    r0, r1 = N - base, N
    for _ in range(50):
        gm.vecchia_partials(THETA, r0, r1)
    ws = []
    for _ in range(reps):
        t0 = time.perf_counter()
        gm.vecchia_partials(THETA, r0, r1)
        ws.append(time.perf_counter() - t0)
    out[f"n{nr}"] = {"rows": [r0, r1], "wall_ms_no_events": float(np.median(ws)) * 1e3}
# the Python-side cost of one call (argument conversion + ctypes), from a zero-row range
ws = []
for _ in range(reps):
    t0 = time.perf_counter()
    gm.vecchia_partials(THETA, N, N)
    ws.append(time.perf_counter() - t0)
out["empty_range_wall_ms"] = float(np.median(ws)) * 1e3
gm.last_kernel_ms()   # from here on evaluations record HIP events
for nr in (1, 2, 4, 8):
    base = N // nr
    r0, r1 = N - base, N
    ws, ks, ss = [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        gm.vecchia_partials(THETA, r0, r1)
        ws.append(time.perf_counter() - t0)
        k = gm.last_kernel_ms()
        ks.append(k[0])
        ss.append(k[1])
    out[f"n{nr}"].update({"wall_ms_events": float(np.median(ws)) * 1e3, "kernel_ms": float(np.median(ks)),
                          "kernel_plus_sum_ms": float(np.median(ss))})
print(json.dumps(out, indent=1))
