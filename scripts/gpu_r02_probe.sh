#!/bin/bash
# GPU box: latent tests, plan timing, then level-kernel probes (GPBOOST_AMD_LEVEL_PROBE 1 / 2:
# timing only, results wrong). Each GPU step time-limited, && chained.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
TAG="${TAG:-r02}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_latent.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/latent_tests_${TAG}.log 2>&1 && \
GPBOOST_AMD_PRECOND_SPLIT=1 PLANS="${PLANS:-2048:14336}" LIKS="${LIKS:-gaussian bernoulli_logit}" \
    timeout -k 10 600 python -u scripts/plan_ab.py > gpurun_out/plan_ab_${TAG}.log 2>&1 && \
GPBOOST_AMD_LEVEL_PROBE=1 GPBOOST_AMD_PRECOND_SPLIT=1 PLANS="2048:14336" LIKS=gaussian \
    timeout -k 10 300 python -u scripts/plan_ab.py > gpurun_out/probe1_${TAG}.log 2>&1 && \
GPBOOST_AMD_LEVEL_PROBE=2 GPBOOST_AMD_PRECOND_SPLIT=1 PLANS="2048:14336" LIKS=gaussian \
    timeout -k 10 300 python -u scripts/plan_ab.py > gpurun_out/probe2_${TAG}.log 2>&1
