#!/bin/bash
# levelT waves-per-row A/B (t = 51 tail levels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MODES=4 GPBOOST_AMD_PRECOND_SPLIT=1 timeout -k 10 300 python -u scripts/head_ab.py > gpurun_out/nw_ab.log 2>&1 || exit $?
MODES=4 GPBOOST_AMD_PRECOND_SPLIT=1 GPBOOST_AMD_LEVELT_NW=2 timeout -k 10 300 python -u scripts/head_ab.py >> gpurun_out/nw_ab.log 2>&1
