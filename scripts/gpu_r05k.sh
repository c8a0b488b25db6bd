#!/bin/bash
# Round-5 GPU run k: reference-draw predictions + order_pred_first elementwise.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
timeout -k 10 900 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_latent_pred_1t.py tests/test_gpu_predict.py > $O/r05k_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed|Error" $O/r05k_tests.log | head -20
exit $rc
