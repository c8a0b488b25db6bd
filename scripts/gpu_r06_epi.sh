#!/bin/bash
# Round 6: batched GEMM epilogue reads (dense + sparse Cholesky), unconditional loads in the front assembly and the
# single-column backward sweep: parity of every path using them, dense / VIF-Laplace / Vecchia-Cholesky timings
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_fitc.py \
  tests/test_gpu_fitc_laplace.py tests/test_gpu_dense_laplace.py tests/test_gpu_vif.py tests/test_gpu_grouped.py \
  tests/test_gpu_latent_chol.py tests/test_gpu_latent_pred.py tests/test_gpu_vif_laplace.py tests/test_gpu_vif_pred.py \
  tests/test_gpu_mode_cap.py tests/test_gpu_predict.py -p no:cacheprovider > gpurun_out/epi_tests.log 2>&1 || { tail -30 gpurun_out/epi_tests.log; exit 1; }
tail -2 gpurun_out/epi_tests.log
timeout -k 10 300 python3 scripts/time_dense.py 20000 > gpurun_out/epi_dense.log 2>&1 || { cat gpurun_out/epi_dense.log; exit 1; }
cat gpurun_out/epi_dense.log
timeout -k 10 300 python3 scripts/vifl_time.py 100000 > gpurun_out/epi_vifl.log 2>&1 || { cat gpurun_out/epi_vifl.log; exit 1; }
tail -10 gpurun_out/epi_vifl.log | cut -c1-160
