#!/bin/bash
# GPU box: latent parity tests, then the plan A/B at n = 100k. Each GPU step time-limited, && chained.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
TAG="${TAG:-r02}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_latent.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/latent_tests_${TAG}.log 2>&1 && \
GPBOOST_AMD_PRECOND_SPLIT=1 PLANS="${PLANS:-0:14336 2048:14336 4096:14336}" LIKS="${LIKS:-gaussian bernoulli_logit}" \
    timeout -k 10 600 python -u scripts/plan_ab.py > gpurun_out/plan_ab_${TAG}.log 2>&1
