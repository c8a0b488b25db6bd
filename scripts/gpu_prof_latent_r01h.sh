#!/bin/bash
# rocprofv3 kernel stats of the default bench including the n=100k latent leg (current tail kernels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_latent_r01h
# hipGraph replay segfaults inside the profiler library under --kernel-trace; launch eagerly (same kernels)
export GPBOOST_AMD_NO_GRAPH=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_latent_r01h" -o lat --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 5 --latent-steps 1 > "$R/gpurun_out/prof_latent_r01h/run.log" 2>&1
