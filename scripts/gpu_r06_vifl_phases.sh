#!/bin/bash
# Round 6: VIF-Laplace per-phase device times (GPBOOST_AMD_TIMING) at n = 100k
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/vifl_time.py 100000 > gpurun_out/vifl_phases.log 2>&1 || { cat gpurun_out/vifl_phases.log; exit 1; }
tail -40 gpurun_out/vifl_phases.log | cut -c1-200
