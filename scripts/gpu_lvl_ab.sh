#!/bin/bash
# tail level kernel shape A/B: t=51 waves per row (1 vs default), t=1 lanes per row (G)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/lvl_ab.log
for cfg in "" "GPBOOST_AMD_LEVELT_NW=1" "GPBOOST_AMD_LEVEL1_G=16" "GPBOOST_AMD_LEVEL1_G=32"; do
  echo "cfg=$cfg" >> gpurun_out/lvl_ab.log
  env $cfg MODES=4 GPBOOST_AMD_PRECOND_SPLIT=1 timeout -k 10 300 python -u scripts/head_ab.py >> gpurun_out/lvl_ab.log 2>&1 || exit $?
done
