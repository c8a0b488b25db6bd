#!/bin/bash
# latent parity suite + timing with the per-solve waves-per-row default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_latent.py -x -q --timeout 300 --timeout-method thread > gpurun_out/nw_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/nw_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
MODES="1 4" LIKS="gaussian bernoulli_logit" GPBOOST_AMD_PRECOND_SPLIT=1 timeout -k 10 300 python -u scripts/head_ab.py > gpurun_out/nw_final.log 2>&1
