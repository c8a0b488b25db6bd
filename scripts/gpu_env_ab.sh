#!/bin/bash
# GPU box: A/B of environment settings on the latent plan timing (plan_ab.py per setting).
#   CFGS="GPBOOST_AMD_LEVELT_FORM=gather GPBOOST_AMD_LEVELT_FORM=chunk" TAG=x bash scripts/gpu_env_ab.sh
# Each CFG is one space-free token of comma-separated VAR=value pairs ("-" = defaults).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
TAG="${TAG:-x}"
OUT=gpurun_out/env_ab_${TAG}.log
: > "$OUT"
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${TEST_FILES:-tests/test_gpu_latent.py} \
    > gpurun_out/env_ab_tests_${TAG}.log 2>&1 || { tail -30 gpurun_out/env_ab_tests_${TAG}.log; exit 1; }
  tail -1 gpurun_out/env_ab_tests_${TAG}.log >> "$OUT"
fi
for cfg in ${CFGS:--}; do
  echo "== $cfg" >> "$OUT"
  envs=()
  [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
  env "${envs[@]}" GPBOOST_AMD_PRECOND_SPLIT=1 PLANS="${PLANS:-2048:14336}" LIKS="${LIKS:-gaussian}" \
      timeout -k 10 300 python -u scripts/plan_ab.py >> "$OUT" 2>&1 || exit 1
done
grep -E "^==|eval=|tail_|seg_|passed|failed" "$OUT"
