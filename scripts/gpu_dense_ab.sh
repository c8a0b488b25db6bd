#!/bin/bash
# GPU box: dense-path timing A/B over in-tree variant builds (gpboost_amd/lib/ab).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG="${TAG:-r02}"
mkdir -p gpurun_out
OUT=gpurun_out/dense_ab_${TAG}.log
: > $OUT
for v in "" ${VARIANTS}; do
  echo "== variant '${v}'" >> $OUT
  GPBOOST_AMD_VARIANT=$v timeout -k 10 240 python scripts/time_dense.py 20000 >> $OUT 2>&1 || exit 1
done
