"""Run bench.py's Cholesky Laplace-Vecchia leg alone: python scripts/chol/bench_leg.py [steps] [--no-cpu]"""
import json
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402
from gpboost_amd import synthetic  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 3
X = synthetic.bench_coords(100_000)
print(json.dumps(bench.bernoulli_chol_leg(X, steps, "--no-cpu" not in sys.argv)), flush=True)
