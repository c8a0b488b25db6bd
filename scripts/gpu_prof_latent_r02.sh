#!/bin/bash
# GPU box: rocprofv3 kernel trace of one latent evaluation (eager launches; the tracer does not
# survive hipGraph replay on this image) summarised on the box (the trace CSV is too large to
# copy back), plus one PMC pass (L2 hit / miss) over the same run. Each step time-limited.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/prof
TAG="${TAG:-r02}"
export GPBOOST_AMD_NO_GRAPH=1
timeout -k 10 300 python -u scripts/prof_latent_one.py > gpurun_out/noprof_${TAG}.log 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$R/gpurun_out/prof/${TAG}" -o lat -- python3 "$R/scripts/prof_latent_one.py" \
    > "$R/gpurun_out/prof_${TAG}.log" 2>&1 ) && \
python scripts/trace_summary.py gpurun_out/prof/${TAG} gpurun_out/trace_${TAG}.txt > /dev/null && \
find gpurun_out/prof/${TAG} -name "*kernel_trace.csv" -delete && \
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d "$R/gpurun_out/prof/${TAG}_pmc" -o l2 -- python3 "$R/scripts/prof_latent_one.py" \
    > "$R/gpurun_out/pmc_${TAG}.log" 2>&1 ) && \
python scripts/pmc_by_kernel.py gpurun_out/prof/${TAG}_pmc gpurun_out/pmc_${TAG}.txt && \
find gpurun_out/prof/${TAG}_pmc -name "*counter_collection.csv" -delete
