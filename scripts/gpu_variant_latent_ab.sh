#!/bin/bash
# GPU box: latent plan timing (plan_ab.py, per-part split) for in-tree library variants
# (GPBOOST_AMD_VARIANT, see gpboost_amd/build.py).  VARIANTS="base r4" TAG=x bash scripts/gpu_variant_latent_ab.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
OUT=gpurun_out/var_ab_${TAG:-x}.log
: > "$OUT"
for v in ${VARIANTS:-base}; do
  echo "== $v" >> "$OUT"
  if [ "$v" = base ]; then vv=""; else vv=$v; fi
  GPBOOST_AMD_VARIANT=$vv GPBOOST_AMD_PRECOND_SPLIT=1 PLANS="${PLANS:-2048:14336}" LIKS="${LIKS:-gaussian}" \
      timeout -k 10 300 python -u scripts/plan_ab.py >> "$OUT" 2>&1 || exit 1
done
grep -E "^==|operator parts|eval=" "$OUT"
