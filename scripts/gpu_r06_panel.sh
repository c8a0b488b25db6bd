#!/bin/bash
# Round 6: single-column sparse solves — single-workgroup level sweeps with all loads of a step in flight; A/B of the
# single-workgroup bound (GPBOOST_AMD_CHOL_SMALL_PANEL) on the VIF-Laplace probe (n = 100k), Cholesky-path parity
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_latent_chol.py \
  tests/test_gpu_vif_laplace.py tests/test_gpu_mode_cap.py tests/test_gpu_latent_pred.py -p no:cacheprovider > gpurun_out/panel_tests.log 2>&1 || { tail -30 gpurun_out/panel_tests.log; exit 1; }
tail -2 gpurun_out/panel_tests.log
for P in 65536 262144 1048576 4194304; do
  GPBOOST_AMD_CHOL_SMALL_PANEL=$P timeout -k 10 300 python3 scripts/vifl_time.py 100000 > gpurun_out/panel_$P.log 2>&1 || { tail -5 gpurun_out/panel_$P.log; exit 1; }
  echo "panel $P: $(grep 'newton solves' gpurun_out/panel_$P.log | tail -1) ; $(grep 'n=100000' gpurun_out/panel_$P.log | cut -c1-80)"
done
