#!/bin/bash
# GPU box: merge depth x waves-per-row A/B of the tail kernels (plan_ab.py per setting, gaussian).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
TAG="${TAG:-r02}"
: > gpurun_out/nw_${TAG}.log
for nw in ${NWS:-1 2}; do
  echo "== NW=$nw" >> gpurun_out/nw_${TAG}.log
  GPBOOST_AMD_LEVELT_NW=$nw GPBOOST_AMD_PRECOND_SPLIT=1 PLANS="${PLANS:-2048:14336:4 2048:14336:8}" LIKS=gaussian \
      timeout -k 10 300 python -u scripts/plan_ab.py >> gpurun_out/nw_${TAG}.log 2>&1 || exit 1
done
