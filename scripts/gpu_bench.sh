#!/bin/bash
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
# GPU-box benchmark + rocprofv3 kernel-trace summary. Each GPU step time-limited, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/prof
TAG="${TAG:-r01}"
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof/${TAG}" -o run -- python "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} \
    > "$R/gpurun_out/prof_${TAG}.log" 2>&1 )
rc=$?
echo "rc=$rc" >> gpurun_out/bench_${TAG}.err
exit $rc
