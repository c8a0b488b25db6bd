#!/bin/bash
# Round 6: the rewritten VIF row kernel (chunked loads, VGPR-form MFMA, two LDS matrices), the spatial processing order
# of the row / B-product kernels: VIF / VIF-Laplace / dense / FITC / sparse Cholesky parity, timings with and
# without the order, a kernel trace of the VIF leg and of the VIF-Laplace n = 100k probe.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vif.py tests/test_gpu_vif_pred.py \
  tests/test_gpu_vif_laplace.py tests/test_gpu_dense.py tests/test_gpu_fitc.py tests/test_gpu_latent_chol.py \
  -p no:cacheprovider > gpurun_out/vifrows_tests.log 2>&1 || { tail -30 gpurun_out/vifrows_tests.log; exit 1; }
tail -3 gpurun_out/vifrows_tests.log
timeout -k 10 200 python3 scripts/time_vif.py 100000 > gpurun_out/vifrows_time.log 2>&1 || { cat gpurun_out/vifrows_time.log; exit 1; }
GPBOOST_AMD_VIF_ORDER=0 timeout -k 10 200 python3 scripts/time_vif.py 100000 > gpurun_out/vifrows_time_noord.log 2>&1 || { cat gpurun_out/vifrows_time_noord.log; exit 1; }
timeout -k 10 300 python3 scripts/vifl_time.py 100000 > gpurun_out/vifl_time.log 2>&1 || { cat gpurun_out/vifl_time.log; exit 1; }
cat gpurun_out/vifrows_time.log gpurun_out/vifrows_time_noord.log gpurun_out/vifl_time.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/vifrows_prof" -o k -- python3 "$R/scripts/time_vif.py" 100000 > "$R/gpurun_out/vifrows_prof.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/vifl_prof" -o k -- python3 "$R/scripts/vifl_time.py" 100000 > "$R/gpurun_out/vifl_prof.log" 2>&1 || exit 1
cd "$R" && for d in vifrows_prof vifl_prof; do f=$(find gpurun_out/$d -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-200; find gpurun_out/$d -name "*kernel_trace.csv" -delete; done
