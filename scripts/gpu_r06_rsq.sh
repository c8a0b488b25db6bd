#!/bin/bash
# Round 6: sparse diagonal blocks with pivot by rsqrt + Newton instead of sqrt + divisions: Cholesky-path parity, VIF-Laplace / Cholesky probes
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_latent_chol.py \
  tests/test_gpu_vif_laplace.py tests/test_gpu_mode_cap.py tests/test_gpu_latent_pred.py -p no:cacheprovider > gpurun_out/rq_tests.log 2>&1 || { tail -30 gpurun_out/rq_tests.log; exit 1; }
tail -2 gpurun_out/rq_tests.log
timeout -k 10 300 python3 scripts/vifl_time.py 100000 > gpurun_out/rq_vifl.log 2>&1 || { tail -5 gpurun_out/rq_vifl.log; exit 1; }
GPBOOST_AMD_TIMING=1 timeout -k 10 300 python3 scripts/chol/time_chol.py 100000 3 > gpurun_out/rq_chol.log 2>&1 || { tail -5 gpurun_out/rq_chol.log; exit 1; }
echo "vifl $(grep '    factor' gpurun_out/rq_vifl.log | tail -1) ; $(grep 'n=100000' gpurun_out/rq_vifl.log | cut -c1-120)"
echo "chol $(grep 'eval 2' gpurun_out/rq_chol.log) $(grep 'latent cholesky' gpurun_out/rq_chol.log | tail -1)"
