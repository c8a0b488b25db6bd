#!/bin/bash
# head-split knobs (K) and a kernel-level profile of the mode-4 preconditioner
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MODES=4 timeout -k 10 200 python -u scripts/head_ab.py > gpurun_out/head_ab2.log 2>&1 || exit $?
MODES=4 GPBOOST_AMD_HEAD_ROWS=16384 timeout -k 10 200 python -u scripts/head_ab.py >> gpurun_out/head_ab2.log 2>&1 || exit $?
MODES=4 GPBOOST_AMD_HEAD_ROWS=8192 timeout -k 10 200 python -u scripts/head_ab.py >> gpurun_out/head_ab2.log 2>&1 || exit $?
MODES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o run -- python -u scripts/head_ab.py > gpurun_out/head_prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/head_prof.log
