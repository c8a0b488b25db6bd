#!/bin/bash
# Round 6: the rewritten VIF row kernel (chunked loads, VGPR-form MFMA, two LDS matrices) and the VGPR-form MFMA
# build: VIF / VIF-Laplace / dense / FITC / sparse Cholesky parity, then timings and a kernel trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vif.py tests/test_gpu_vif_pred.py \
  tests/test_gpu_vif_laplace.py tests/test_gpu_dense.py tests/test_gpu_fitc.py tests/test_gpu_latent_chol.py \
  -p no:cacheprovider > gpurun_out/vifrows_tests.log 2>&1 || { tail -30 gpurun_out/vifrows_tests.log; exit 1; }
tail -3 gpurun_out/vifrows_tests.log
timeout -k 10 200 python3 scripts/time_vif.py 100000 > gpurun_out/vifrows_time.log 2>&1 || { cat gpurun_out/vifrows_time.log; exit 1; }
cat gpurun_out/vifrows_time.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/vifrows_prof" -o k -- python3 "$R/scripts/time_vif.py" 100000 > "$R/gpurun_out/vifrows_prof.log" 2>&1 || exit 1
cd "$R" && f=$(find gpurun_out/vifrows_prof -name "*kernel_stats.csv" | head -1) && head -14 "$f"
