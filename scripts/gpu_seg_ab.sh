#!/bin/bash
# A/B of the segmented B^T (t = 1) kernel shape: in-tree library variants (gpboost_amd/build.py,
# GPBOOST_AMD_VARIANT) timed by GPB_BenchLatentOperators at n = 100k (operator parts).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/seg_ab
mkdir -p $O
for v in ${VARIANTS:-base u8 e256 u2e128}; do
  if [ "$v" = base ]; then export GPBOOST_AMD_VARIANT=; else export GPBOOST_AMD_VARIANT=$v; fi
  for rep in 1 2 3; do
    GPBOOST_AMD_PRECOND_SPLIT=1 timeout -k 10 200 python -u scripts/prof_op1.py > $O/op_${v}_$rep.log 2>&1 || exit $?
    echo "$v $rep $(grep 'operator parts' $O/op_${v}_$rep.log | tr '\n' ' ')" >> $O/summary.log
  done
done
cat $O/summary.log
