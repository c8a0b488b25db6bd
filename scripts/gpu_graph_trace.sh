#!/bin/bash
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
# GPU box: does rocprofv3 --kernel-trace survive the latent path's hipGraph replay (the default
# launch path)? One profiled latent evaluation without GPBOOST_AMD_NO_GRAPH; the exit status and
# the log tail go to gpurun_out/graph_trace/result.txt. Run it LAST in a call (a crash ends the call).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/graph_trace
( cd /tmp && export TMPDIR=/tmp N=20000 && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/graph_trace/prof" -o lat -- python3 "$R/scripts/prof_latent_one.py" \
    > "$R/gpurun_out/graph_trace/run.log" 2>&1 )
rc=$?
{ echo "exit status: $rc"; tail -30 "$R/gpurun_out/graph_trace/run.log"; } > "$R/gpurun_out/graph_trace/result.txt"
exit $rc
