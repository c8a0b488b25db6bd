#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
MODES=4 GPBOOST_AMD_PRECOND_SPLIT=1 timeout -k 10 200 python -u scripts/head_ab.py > gpurun_out/head_ab3.log 2>&1 || exit $?
MODES=4 GPBOOST_AMD_PRECOND_SPLIT=1 GPBOOST_AMD_HEAD_ROWS=4096 timeout -k 10 200 python -u scripts/head_ab.py >> gpurun_out/head_ab3.log 2>&1
