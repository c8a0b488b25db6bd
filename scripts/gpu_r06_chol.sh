#!/bin/bash
# Round 6: sparse Cholesky small-launch GEMM form (K <= 64, single-shot loads): Cholesky-path parity, VIF-Laplace timing
# with and without it, a trace of the VIF-Laplace probe (busy vs wall, per-kernel totals)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_latent_chol.py \
  tests/test_gpu_vif_laplace.py tests/test_gpu_mode_cap.py -p no:cacheprovider > gpurun_out/chol_tests.log 2>&1 || { tail -30 gpurun_out/chol_tests.log; exit 1; }
tail -2 gpurun_out/chol_tests.log
timeout -k 10 300 python3 scripts/vifl_time.py 100000 > gpurun_out/chol_vifl_time.log 2>&1 || { cat gpurun_out/chol_vifl_time.log; exit 1; }
GPBOOST_AMD_CHOL_K64=0 timeout -k 10 300 python3 scripts/vifl_time.py 100000 > gpurun_out/chol_vifl_time_nok64.log 2>&1 || { cat gpurun_out/chol_vifl_time_nok64.log; exit 1; }
grep "n=" gpurun_out/chol_vifl_time.log gpurun_out/chol_vifl_time_nok64.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/chol_vifl_prof" -o k -- python3 "$R/scripts/vifl_time.py" 100000 > "$R/gpurun_out/chol_vifl_prof.log" 2>&1 || exit 1
cd "$R" && python3 scripts/trace_gaps.py gpurun_out/chol_vifl_prof > gpurun_out/chol_vifl_gaps.txt && cat gpurun_out/chol_vifl_gaps.txt
find gpurun_out/chol_vifl_prof -name "*kernel_trace.csv" -size +20M -delete
