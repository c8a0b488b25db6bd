"""Debug probe: VIF Laplace gradient with fixed effects, GPU vs the dense restatement (poisson, n = 1000)."""
import sys

import numpy as np

sys.path.insert(0, ".")
from gpboost_amd import synthetic  # noqa: E402

n, m, nn = 1000, 30, 10
X = synthetic.bench_coords(n)
y = synthetic.bench_poisson_y(X)
fe = 0.3 * np.sin(3.0 * X[:, 0]) - 0.2
cp = [0.9, 0.12]
if sys.argv[1] == "gpu":
    from gpboost_amd import GPModel
    for f in (None, fe, 0.0 * fe):
        gm = GPModel(gp_coords=X, likelihood="poisson", gp_approx="full_scale_vecchia", num_ind_points=m,
                     cov_function="exponential", num_neighbors=nn, seed=0, matrix_inversion_method="cholesky")
        print("GPU", gm.neg_log_likelihood_and_grad(cp, y, fixed_effects=f), flush=True)
else:
    from oracle import oracle as O
    from oracle.vif_laplace_oracle import VifLaplaceOracle
    perm, Z, _ = O.vif_inducing_points(X, m, "kmeans++", 0, True)
    xv = X[perm]
    nb = O.find_neighbors(xv, nn)
    tr = O.transform_latent(0, cp)
    for f in (None, fe):
        o = VifLaplaceOracle(xv, y[perm], nb, Z, 0, tr[0], tr[1], "poisson", fixed_effects=None if f is None else f[perm])
        print("ORACLE", o.nll, o.grad()[0])
