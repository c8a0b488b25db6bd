#!/bin/bash
# GPU box: rocprofv3 kernel trace of one latent evaluation (eager launches), plus the same run
# without the profiler for the wall time. Each step time-limited, && chained.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/prof
TAG="${TAG:-r02}"
GPBOOST_AMD_NO_GRAPH=1 timeout -k 10 300 python -u scripts/prof_latent_one.py > gpurun_out/noprof_${TAG}.log 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && GPBOOST_AMD_NO_GRAPH=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$R/gpurun_out/prof/${TAG}" -o lat -- python3 "$R/scripts/prof_latent_one.py" \
    > "$R/gpurun_out/prof_${TAG}.log" 2>&1 ) && \
python scripts/trace_summary.py gpurun_out/prof/${TAG} gpurun_out/trace_${TAG}.txt > /dev/null && \
find gpurun_out/prof/${TAG} -name "*kernel_trace.csv" -delete
