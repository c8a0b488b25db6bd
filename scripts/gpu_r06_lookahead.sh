#!/bin/bash
# Round 6: sparse Cholesky factorization with one block of lookahead on two streams: Cholesky-path parity, timings of
# the VIF-Laplace and Cholesky Laplace-Vecchia probes with and without it (GPBOOST_AMD_CHOL_LOOKAHEAD=0)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_latent_chol.py \
  tests/test_gpu_vif_laplace.py tests/test_gpu_mode_cap.py tests/test_gpu_latent_pred.py -p no:cacheprovider > gpurun_out/la_tests.log 2>&1 || { tail -30 gpurun_out/la_tests.log; exit 1; }
tail -2 gpurun_out/la_tests.log
for V in 1 0; do
  GPBOOST_AMD_CHOL_LOOKAHEAD=$V timeout -k 10 300 python3 scripts/vifl_time.py 100000 > gpurun_out/la_vifl_$V.log 2>&1 || { tail -5 gpurun_out/la_vifl_$V.log; exit 1; }
  GPBOOST_AMD_CHOL_LOOKAHEAD=$V GPBOOST_AMD_TIMING=1 timeout -k 10 300 python3 scripts/chol/time_chol.py 100000 3 > gpurun_out/la_chol_$V.log 2>&1 || { tail -5 gpurun_out/la_chol_$V.log; exit 1; }
  echo "lookahead $V: vifl $(grep '    factor' gpurun_out/la_vifl_$V.log | tail -1) ; $(grep 'n=100000' gpurun_out/la_vifl_$V.log | cut -c1-60) ; chol $(grep 'eval 2' gpurun_out/la_chol_$V.log) $(grep 'latent cholesky' gpurun_out/la_chol_$V.log | tail -1)"
done
