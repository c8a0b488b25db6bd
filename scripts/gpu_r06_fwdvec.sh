#!/bin/bash
# Round 6: fused single-column forward block steps (kOpFwdVec): Cholesky-path parity, VIF-Laplace phases on / off
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_latent_chol.py \
  tests/test_gpu_vif_laplace.py tests/test_gpu_mode_cap.py tests/test_gpu_latent_pred.py -p no:cacheprovider > gpurun_out/fwdvec_tests.log 2>&1 || { tail -30 gpurun_out/fwdvec_tests.log; exit 1; }
tail -2 gpurun_out/fwdvec_tests.log
for V in 1 0; do
  GPBOOST_AMD_CHOL_FWDVEC=$V timeout -k 10 300 python3 scripts/vifl_time.py 100000 > gpurun_out/fwdvec_$V.log 2>&1 || { tail -5 gpurun_out/fwdvec_$V.log; exit 1; }
  echo "fwdvec $V: $(grep 'newton solves' gpurun_out/fwdvec_$V.log | tail -1) ; $(grep 'n=100000' gpurun_out/fwdvec_$V.log | cut -c1-90)"
done
