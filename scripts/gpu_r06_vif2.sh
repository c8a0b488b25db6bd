#!/bin/bash
# Round 6: VIF row kernel with LDS-staged coordinates (tests + timing), and a kernel trace of the dense path (n = 20000)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vif.py tests/test_gpu_vif_pred.py \
  tests/test_gpu_vif_laplace.py -p no:cacheprovider > gpurun_out/vif2_tests.log 2>&1 || { tail -30 gpurun_out/vif2_tests.log; exit 1; }
tail -2 gpurun_out/vif2_tests.log
timeout -k 10 200 python3 scripts/time_vif.py 100000 > gpurun_out/vif2_time.log 2>&1 || { cat gpurun_out/vif2_time.log; exit 1; }
cat gpurun_out/vif2_time.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/vif2_prof" -o k -- python3 "$R/scripts/time_vif.py" 100000 > "$R/gpurun_out/vif2_prof.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/dense_prof" -o k -- python3 "$R/scripts/time_dense.py" 20000 > "$R/gpurun_out/dense_prof.log" 2>&1 || exit 1
cd "$R" && for d in vif2_prof dense_prof; do f=$(find gpurun_out/$d -name "*kernel_stats.csv" | head -1); head -16 "$f" | cut -c1-160; done
python3 scripts/trace_gaps.py gpurun_out/dense_prof > gpurun_out/dense_gaps.txt && cat gpurun_out/dense_gaps.txt
find gpurun_out/vif2_prof gpurun_out/dense_prof -name "*kernel_trace.csv" -size +20M -delete
