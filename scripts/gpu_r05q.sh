#!/bin/bash
# Round-5 GPU run o: grouped cholesky predictive variances.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_grouped.py > $O/r05q_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed|Error|ACTUAL|DESIRED|assert" $O/r05q_tests.log | head -40
exit $rc
