#!/bin/bash
# latent GPU tests with the multi-row t=1 SpMV, then old/new operator timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_latent.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/spmv1_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/spmv1_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
MODES=4 LIKS="gaussian bernoulli_logit" timeout -k 10 300 python -u scripts/head_ab.py > gpurun_out/spmv1_ab.log 2>&1 || exit $?
MODES=4 LIKS="gaussian" GPBOOST_AMD_SPMV1_OLD=1 timeout -k 10 300 python -u scripts/head_ab.py >> gpurun_out/spmv1_ab.log 2>&1
