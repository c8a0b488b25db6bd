#!/bin/bash
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
# GPU box: kernel-trace summary of the dense path (n = 20000, eager launches).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG="${TAG:-r02}"
mkdir -p gpurun_out/prof_dense
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof_dense/${TAG}" -o d -- python3 "$R/scripts/time_dense.py" ${DENSE_N:-20000} \
    > "$R/gpurun_out/prof_dense_${TAG}.log" 2>&1 ) || exit 1
find "gpurun_out/prof_dense/${TAG}" -name "*kernel_trace.csv" -delete
