"""One measured reference dense evaluation at BASELINE config 2's size (n = 20000, exponential, L-BFGS unit:
nll + gradient, sigma^2 profiled) on the GPU box's host cores, for bench.py's dense cpu_baseline (in place of
the n^3 extrapolation from n = 4000). Runs oracle/_ref/ref_harness (the reference compiled from its sources);
prints a progress line every 30 s. Output: gpurun_out/ref_dense_n20000.json."""
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gpboost_amd import synthetic  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
X = synthetic.bench_coords(n)
Y = synthetic.bench_gaussian_y(n)
with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
    f.write(np.array([n, 2], dtype=np.int32).tobytes())
    f.write(np.ascontiguousarray(X.T).tobytes())
    f.write(np.ascontiguousarray(Y).tobytes())
    path = f.name
done = threading.Event()
t0 = time.time()


def tick():
    while not done.wait(30):
        print(f"[ref dense n={n}] {time.time() - t0:.0f} s", flush=True)


threading.Thread(target=tick, daemon=True).start()
out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_harness"), path, "cov_fct=exponential", "gp_approx=none",
                      "mode=lbfgs", "reps=1", "cov_pars=0.1,1.0,0.1"], capture_output=True, text=True, timeout=1100,
                     env=dict(os.environ, OMP_NUM_THREADS=str(threads)), check=True)
done.set()
os.unlink(path)
r = json.loads(out.stdout)
rec = {"n": n, "threads": threads, "median_time_s": r["median_time"], "nll": r["nll"], "grad": r["grad"],
       "wall_s": time.time() - t0, "nproc": os.cpu_count(), "kind": "reference",
       "what": "one dense L-BFGS-unit evaluation (nll + gradient, sigma^2 profiled) of the reference"}
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", f"ref_dense_n{n}.json"), "w") as f:
    json.dump(rec, f, indent=1)
print(json.dumps(rec))
