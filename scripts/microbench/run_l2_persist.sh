#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/mb
timeout -k 10 60 scripts/microbench/l2_persist > gpurun_out/mb/l2_persist.log 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv \
    -d "$R/gpurun_out/mb/pmc" -o l2 -- "$R/scripts/microbench/l2_persist" >> "$R/gpurun_out/mb/l2_persist.log" 2>&1 )
