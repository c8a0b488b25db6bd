#!/bin/bash
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
# GPU box: the round's profile set for the current kernels — row-kernel HBM traffic passes
# (gpu_pmc_rows_traffic.sh), row-kernel SQ passes (gpu_pmc_rows.sh) and a rocprofv3 kernel trace of
# the full bench with the latent preconditioner launched eagerly (GPBOOST_AMD_NO_GRAPH=1: under
# --kernel-trace the hipGraph replay segfaults inside the tracer, profiles/r03/rocprof_graph_crash_r03j.log).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG="${TAG:-r03}"
mkdir -p gpurun_out/prof
TAG=$TAG bash scripts/gpu_pmc_rows_traffic.sh > gpurun_out/pmc_traffic_${TAG}.log 2>&1 || exit 1
TAG=$TAG bash scripts/gpu_pmc_rows.sh || exit 1
( cd /tmp && export TMPDIR=/tmp && GPBOOST_AMD_NO_GRAPH=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof/${TAG}" -o run -- python "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline \
    > "$R/gpurun_out/prof_${TAG}.log" 2>&1 ) || exit 1
# keep the summaries only (the full per-dispatch trace of the latent legs is hundreds of MB)
find gpurun_out/prof/${TAG} -name '*kernel_trace*' -delete
find gpurun_out/pmc_rows gpurun_out/pmc_traffic -name '*counter_collection*' -size +20M -delete
du -sh gpurun_out
