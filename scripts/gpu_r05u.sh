#!/bin/bash
# Round-5 GPU run u: internal optimizers (gradient descent, Fisher scoring) beside the optimizer / grouped / combined suites.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_internal_optim.py tests/test_gpu_optim.py tests/test_gpu_grouped.py tests/test_gpu_combined.py \
  > $O/r05u_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed|Error|ACTUAL|DESIRED|assert" $O/r05u_tests.log | head -40
exit $rc
