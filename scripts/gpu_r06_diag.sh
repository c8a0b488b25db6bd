#!/bin/bash
# Round 6: four-wave right-looking inverse of the dense diagonal blocks (bit-identical by construction): dense /
# FITC / VIF / grouped-cholesky parity, dense n = 20000 timing with a kernel trace
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_fitc.py \
  tests/test_gpu_fitc_laplace.py tests/test_gpu_dense_laplace.py tests/test_gpu_vif.py tests/test_gpu_grouped.py \
  tests/test_gpu_latent_chol.py tests/test_gpu_latent_pred.py tests/test_gpu_vif_laplace.py \
  -p no:cacheprovider > gpurun_out/diag_tests.log 2>&1 || { tail -30 gpurun_out/diag_tests.log; exit 1; }
tail -2 gpurun_out/diag_tests.log
timeout -k 10 300 python3 scripts/time_dense.py 20000 > gpurun_out/diag_dense_time.log 2>&1 || { cat gpurun_out/diag_dense_time.log; exit 1; }
cat gpurun_out/diag_dense_time.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/diag_prof" -o k -- python3 "$R/scripts/time_dense.py" 20000 > "$R/gpurun_out/diag_prof.log" 2>&1 || exit 1
cd "$R" && python3 scripts/trace_gaps.py gpurun_out/diag_prof > gpurun_out/diag_gaps.txt && cat gpurun_out/diag_gaps.txt
find gpurun_out/diag_prof -name "*kernel_trace.csv" -size +20M -delete
