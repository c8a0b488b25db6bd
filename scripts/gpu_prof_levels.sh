#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/prof_levels"
cd /tmp && export TMPDIR=/tmp
GPBOOST_AMD_NO_GRAPH=1 timeout -k 10 600 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_levels" -o run --output-format csv -- python3 "$R/scripts/prof_latent_one.py" gaussian 100000 4 > "$R/gpurun_out/prof_levels/run.log" 2>&1
