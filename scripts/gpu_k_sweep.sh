#!/bin/bash
# head size K sweep with the current head kernel (gaussian t=51 and bernoulli t=50/1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/k_sweep.log
for K in 12288 14336 16384; do
  echo "K=$K" >> gpurun_out/k_sweep.log
  MODES=4 LIKS="gaussian bernoulli_logit" GPBOOST_AMD_HEAD_ROWS=$K timeout -k 10 300 python -u scripts/head_ab.py >> gpurun_out/k_sweep.log 2>&1 || exit $?
done
