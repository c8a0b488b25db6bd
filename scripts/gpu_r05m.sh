#!/bin/bash
# Round-5 GPU run m: Vecchia Fisher pieces vs the oracle, then the std dev tests.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 -u scripts/diag_fisher.py 500 10 > $O/r05m_diag.log 2>&1 &&
timeout -k 10 300 python3 -u scripts/diag_fisher.py 3000 20 >> $O/r05m_diag.log 2>&1
rc=$?
cat $O/r05m_diag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_stddev_vecchia.py > $O/r05m_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed|Error|ACTUAL|DESIRED" $O/r05m_tests.log | head -30
exit $rc
