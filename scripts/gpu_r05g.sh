#!/bin/bash
# Round-5 GPU run g: full-scale Vecchia (VIF) parity.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_vif.py \
  > $O/r05g_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error|assert" $O/r05g_tests.log | head -60
exit $rc
