"""Diagnostics (GPU box): the Vecchia Fisher-information pieces (GPBOOST_AMD_FISHER_DUMP) against the CPU
restatement (oracle/vecchia_fisher_oracle.py), piece by piece. Usage: python3 scripts/diag_fisher.py [n nn]"""
import os
import sys
import tempfile

import numpy as np
from scipy.sparse.linalg import spsolve_triangular

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpboost_amd import GPModel, synthetic  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle.vecchia_fisher_oracle import vecchia_factor_orig  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
nn = int(sys.argv[2]) if len(sys.argv) > 2 else 10
t = 8
cp = [0.25, 1.0, 0.1]
X = synthetic.bench_coords(n)
y = synthetic.bench_spatial_gaussian_y(X)
path = os.path.join(tempfile.gettempdir(), "fisher_dump.bin")
os.environ["GPBOOST_AMD_FISHER_DUMP"] = path
gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=nn, seed=0)
gm.set_optim_params({"num_rand_vec_trace": t})
gm.neg_log_likelihood(cp, y)
sd = gm.get_cov_pars(std_err=True)[1]
raw = np.fromfile(path)
n_, m, t_ = (int(v) for v in raw[:3])
off = 3
def take(cnt, shape):
    global off
    a = raw[off:off + cnt].reshape(shape)
    off += cnt
    return a
Bv, dB0, dB1 = (take(n * m, (n, m)) for _ in range(3))
Do, dD0, dD1 = (take(n, (n,)) for _ in range(3))
Z, P, W, G0, G1, G2 = (take(n * t, (n, t)) for _ in range(6))

_, xv, nb = O.vecchia_setup(X, nn, 0, True)
B, D, dB, dD = vecchia_factor_orig(xv, nb, 0, cp)
def rows(S):
    out = np.zeros((n, m))
    S = S.tocsr()
    for i in range(n):
        for r in range(min(i, m)):
            out[i, r] = S[i, nb[i, r]]
    return out
def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))
print("B", rel(Bv, rows(B)), "Do", rel(Do, 1. / D))
print("dB0", rel(dB0, rows(dB[0])), "dD0", rel(dD0, dD[0]))
print("dB1", rel(dB1, rows(dB[1])), "dD1", rel(dD1, dD[1]))
z = O.gen_probes(n, t, 1, 0)
print("Z", rel(Z, z))
BT = B.T.tocsr()
Wr = spsolve_triangular(BT, z, lower=False)
Sz = spsolve_triangular(B, D[:, None] * Wr, lower=True)
print("P", rel(P, Sz), "W", rel(W, Wr))
g0 = BT @ ((1. / D)[:, None] * (B @ z))
print("G0", rel(G0, g0))
for k, Gk in enumerate((G1, G2)):
    u = -(dB[k] @ Sz) + dD[k][:, None] * Wr
    gk = BT @ ((1. / D)[:, None] * u) - dB[k].T @ Wr
    print(f"G{k + 1}", rel(Gk, gk))
print("sd", sd)
