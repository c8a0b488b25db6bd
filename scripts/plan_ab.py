"""A/B of the VADU preconditioner plan split (vadu_precond.h) on the latent Vecchia path at
n = 100k: per plan "K0:K[:g[:budget]]" (dense head rows : head rows incl. the dense ones : at most g tail levels and
`budget` entries per launch; empty = default) one warm-up and
two timed nll+grad evaluations, the preconditioner's per-application time (t = 51 and t = 1,
GPB_BenchLatentOperators, with the per-step split when GPBOOST_AMD_PRECOND_SPLIT is set), and
the results (they must agree across plans to rounding)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402

n = int(os.environ.get("N", "100000"))
plans = os.environ.get("PLANS", "0:14336 2048:14336").split()
liks = os.environ.get("LIKS", "gaussian").split()
X = synthetic.bench_coords(n)
for lik in liks:
    y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
    for plan in plans:
        k0, k, g, budget = (plan.split(":") + ["", "", "", ""])[:4]
        for name, v in (("DENSE_ROWS", k0), ("HEAD_ROWS", k), ("TAIL_MERGE", g), ("TAIL_BUDGET", budget)):
            if v:
                os.environ["GPBOOST_AMD_" + name] = v
            else:
                os.environ.pop("GPBOOST_AMD_" + name, None)
        gm = GPModel(gp_coords=X, likelihood=lik, cov_function="exponential",
                     gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia", num_neighbors=30,
                     vecchia_ordering="random", seed=0, matrix_inversion_method="iterative")
        p = dict(num_rand_vec_trace=50)
        if lik == "gaussian":
            p["init_aux_pars"] = [0.1]
        gm.set_optim_params(p)
        t0 = time.time()
        r = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
        t1 = time.time()
        ts = []
        for _ in range(2):
            s = time.time()
            r = gm.neg_log_likelihood_and_grad([1.0, 0.1], None)
            ts.append(time.time() - s)
        info = gm.last_iteration_info()
        t = 51 if lik == "gaussian" else 50
        ops = gm.bench_latent_operators(t, 10)
        ops1 = gm.bench_latent_operators(1, 10)
        print(f"{lik} plan={plan} first={t1 - t0:.3f}s eval={np.median(ts):.4f}s nll={r[0]:.12g} grad={r[1]} "
              f"info={info} A_ms(t={t})={ops[0]:.4f} P_ms(t={t})={ops[1]:.4f} launches={ops[3]:.0f} "
              f"A_ms(1)={ops1[0]:.4f} P_ms(1)={ops1[1]:.4f}", flush=True)
        del gm
