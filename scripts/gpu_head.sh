#!/bin/bash
# latent GPU tests, then the preconditioner A/B at n=100k (stops after a crash / time limit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_latent.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/head_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/head_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u scripts/head_ab.py > gpurun_out/head_ab.log 2>&1
rc=$?
echo "ab rc=$rc" >> gpurun_out/head_ab.log
exit $rc
