#!/bin/bash
# Round 6: Cholesky GEMM tile k step 16 vs 32 (GPBOOST_AMD_CHOL_GK=32), batched split-K reduce: Cholesky-path parity
# (both k steps), VIF-Laplace / Cholesky probes
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
T="tests/test_gpu_latent_chol.py tests/test_gpu_vif_laplace.py tests/test_gpu_mode_cap.py tests/test_gpu_latent_pred.py"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $T -p no:cacheprovider > gpurun_out/gk_tests.log 2>&1 || { tail -30 gpurun_out/gk_tests.log; exit 1; }
tail -1 gpurun_out/gk_tests.log
GPBOOST_AMD_CHOL_GK=32 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $T -p no:cacheprovider > gpurun_out/gk32_tests.log 2>&1 || { tail -30 gpurun_out/gk32_tests.log; exit 1; }
tail -1 gpurun_out/gk32_tests.log
for g in 16 32 16 32; do
  GPBOOST_AMD_CHOL_GK=$g timeout -k 10 300 python3 scripts/vifl_time.py 100000 > gpurun_out/gk_vifl$g.log 2>&1 || { tail -5 gpurun_out/gk_vifl$g.log; exit 1; }
  GPBOOST_AMD_CHOL_GK=$g GPBOOST_AMD_TIMING=1 timeout -k 10 300 python3 scripts/chol/time_chol.py 100000 3 > gpurun_out/gk_chol$g.log 2>&1 || { tail -5 gpurun_out/gk_chol$g.log; exit 1; }
  echo "gk=$g vifl $(grep '    factor' gpurun_out/gk_vifl$g.log | tail -1) ; $(grep 'n=100000' gpurun_out/gk_vifl$g.log | cut -c1-80)"
  echo "gk=$g chol $(grep 'latent cholesky' gpurun_out/gk_chol$g.log | tail -1)"
done
