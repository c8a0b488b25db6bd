#!/bin/bash
# Single-vector operator env A/B: latent GPU tests, then GPB_BenchLatentOperators(t = 1) parts at
# n = 100k, three runs per setting. SETTINGS: space-separated NAME=VALUE env assignments
# ("-" = defaults).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/op1_env
mkdir -p $O
: > $O/summary.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_latent.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)" >> $O/summary.log
case $rc in 0|1) ;; *) exit $rc ;; esac
for st in ${SETTINGS:--}; do
  for rep in 1 2 3; do
    if [ "$st" = "-" ]; then
      GPBOOST_AMD_PRECOND_SPLIT=1 timeout -k 10 200 python -u scripts/prof_op1.py > $O/op.log 2>&1 || exit $?
    else
      env "$st" GPBOOST_AMD_PRECOND_SPLIT=1 timeout -k 10 200 python -u scripts/prof_op1.py > $O/op.log 2>&1 || exit $?
    fi
    echo "$st $rep $(grep 'operator parts' $O/op.log | tr '\n' ' ') $(grep '^\[' $O/op.log | grep -v parts)" >> $O/summary.log
  done
done
cat $O/summary.log
exit $rc
