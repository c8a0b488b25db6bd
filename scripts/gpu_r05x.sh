#!/bin/bash
# round 5: covariate-aware internal optimizers (Fisher scoring + wls) on the GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_internal_optim.py \
  tests/test_gpu_covariates.py -m gpu > gpurun_out/tests_r05_wls.log 2>&1
rc=$?
tail -25 gpurun_out/tests_r05_wls.log
exit $rc
