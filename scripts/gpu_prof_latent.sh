#!/bin/bash
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_latent
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_latent" -o lat --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/prof_latent_one.py" gaussian 20000 > "$GRAFT_REPO_ROOT/gpurun_out/prof_latent/run.log" 2>&1
