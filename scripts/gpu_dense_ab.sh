#!/bin/bash
# dense-path GPU tests with the 128x128 GEMM, then timing new vs 64x64-only
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dense_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/dense_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u scripts/time_dense.py > gpurun_out/dense_ab.log 2>&1 || exit $?
GPBOOST_AMD_DIAG_OLD=1 timeout -k 10 300 python -u scripts/time_dense.py >> gpurun_out/dense_ab.log 2>&1
