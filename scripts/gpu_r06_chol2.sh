#!/bin/bash
# Round 6: one forward + one backward sweep per Woodbury solve (VIF-Laplace), fsolve1 in forward-only sweeps:
# Cholesky-path parity (latent Cholesky, VIF-Laplace, predictions), VIF-Laplace phase times
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_latent_chol.py \
  tests/test_gpu_vif_laplace.py tests/test_gpu_mode_cap.py tests/test_gpu_latent_pred.py -p no:cacheprovider > gpurun_out/chol2_tests.log 2>&1 || { tail -30 gpurun_out/chol2_tests.log; exit 1; }
tail -2 gpurun_out/chol2_tests.log
timeout -k 10 300 python3 scripts/vifl_time.py 100000 > gpurun_out/chol2_phases.log 2>&1 || { cat gpurun_out/chol2_phases.log; exit 1; }
tail -12 gpurun_out/chol2_phases.log | cut -c1-200
