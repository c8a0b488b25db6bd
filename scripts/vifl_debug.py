"""Debug probe: VIF Laplace components on the GPU vs the dense restatement (n = 300)."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
os.environ["GPBOOST_AMD_VIFL_DEBUG"] = "1"
from gpboost_amd import GPModel, synthetic  # noqa: E402

n, m, nn = 300, 15, 8
X = synthetic.bench_coords(n)
y = synthetic.bench_bernoulli_y(X)
if sys.argv[1] == "gpu":
    gm = GPModel(gp_coords=X, likelihood="bernoulli_logit", gp_approx="full_scale_vecchia", num_ind_points=m, cov_function="exponential",
                 num_neighbors=nn, seed=1, matrix_inversion_method="cholesky")
    print("GPU", gm.neg_log_likelihood_and_grad([0.7, 0.2], y), flush=True)
    print("GPU Z", gm.inducing_points()[:3].ravel().tolist())
else:
    from oracle import oracle as O
    from oracle.vif_laplace_oracle import VifLaplaceOracle, _logdet
    perm, Z, _ = O.vif_inducing_points(X, m, "kmeans++", 1, True)
    xv = X[perm]
    nb = O.find_neighbors(xv, nn)
    tr = O.transform_latent(0, (0.7, 0.2))
    o = VifLaplaceOracle(xv, y[perm], nb, Z, 0, tr[0], tr[1], "bernoulli_logit")
    A = o.R + np.diag(o.w)
    print("ORACLE D[0..4]", o.D[:5])
    print("ORACLE Z", Z[:3].ravel().tolist(), "trafo", tr)
    print("ORACLE its?", "obj", o.obj, "logdet A", _logdet(A), "sum log Dinv", np.log(o.Dinv).sum(), "logdet Ks",
          _logdet(o.f["Ks"]), "logdet M", _logdet(o.M), "logdet M2", _logdet(o.M2), "nll", o.nll, "grad", o.grad()[0])
