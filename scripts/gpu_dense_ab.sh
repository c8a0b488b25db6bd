#!/bin/bash
# GPU box: dense-path timing A/B over in-tree variant builds (gpboost_amd/lib/ab) and env switches.
# VARIANTS="name env:VAR=1 ..." (a bare name selects libgpboost_amd_<name>.so).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG="${TAG:-r02}"
N="${DENSE_N:-20000}"
mkdir -p gpurun_out
OUT=gpurun_out/dense_ab_${TAG}.log
: > $OUT
for v in "" ${VARIANTS}; do
  echo "== variant '${v}'" >> $OUT
  if [[ "$v" == env:* ]]; then
    env "${v#env:}" timeout -k 10 240 python scripts/time_dense.py $N >> $OUT 2>&1 || exit 1
  else
    GPBOOST_AMD_VARIANT=$v timeout -k 10 240 python scripts/time_dense.py $N >> $OUT 2>&1 || exit 1
  fi
done
