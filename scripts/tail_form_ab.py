"""A/B of the VADU tail solve form at n = 100k (latent Gaussian Vecchia, t = 51): per entry of FORMS
("launch" = one launch per merged level, "persist:W[:g]" = the persistent kernel with W workgroups per
XCD group and g levels per merged level) one warm-up and two timed nll+grad evaluations, the
preconditioner's time per application (GPB_BenchLatentOperators; per-part split with
GPBOOST_AMD_PRECOND_SPLIT=1) and the results (equal to rounding across forms)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402

n = int(os.environ.get("N", "100000"))
forms = os.environ.get("FORMS", "launch persist:64").split()
X = synthetic.bench_coords(n)
y = synthetic.bench_gaussian_y(n)
for form in forms:
    f = form.split(":")
    os.environ["GPBOOST_AMD_TAIL_FORM"] = f[0]
    for k, v in (("GPBOOST_AMD_TAIL_W", f[1] if len(f) > 1 else ""), ("GPBOOST_AMD_TAIL_MERGE", f[2] if len(f) > 2 else "")):
        if v:
            os.environ[k] = v
        else:
            os.environ.pop(k, None)
    gm = GPModel(gp_coords=X, likelihood="gaussian", cov_function="exponential", gp_approx="vecchia_latent",
                 num_neighbors=30, vecchia_ordering="random", seed=0, matrix_inversion_method="iterative")
    gm.set_optim_params(dict(num_rand_vec_trace=50, init_aux_pars=[0.1]))
    t0 = time.time()
    r = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
    t1 = time.time()
    ts = []
    for _ in range(2):
        s = time.time()
        r = gm.neg_log_likelihood_and_grad([1.0, 0.1], None)
        ts.append(time.time() - s)
    ops = gm.bench_latent_operators(51, 20)
    print(f"form={form} first={t1 - t0:.3f}s eval={np.median(ts):.4f}s nll={r[0]:.15g} grad={r[1]} "
          f"info={gm.last_iteration_info()} A_ms={ops[0]:.4f} P_ms={ops[1]:.4f} launches={ops[3]:.0f}", flush=True)
    del gm
