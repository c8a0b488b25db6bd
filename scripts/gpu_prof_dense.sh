#!/bin/bash
# kernel-level profile of the dense path at n=20000 (one warm-up + 3 evaluations)
mkdir -p "$GRAFT_REPO_ROOT/gpurun_out/prof_dense"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_dense" -o dense --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/time_dense.py" 20000 > "$GRAFT_REPO_ROOT/gpurun_out/prof_dense/run.log" 2>&1
