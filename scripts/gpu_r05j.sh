#!/bin/bash
# Round-5 GPU run j: Laplace predictive moments with the reference's one-thread draws; prediction suites.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
timeout -k 10 900 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_latent_pred_1t.py > $O/r05j_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error|assert|Mismatch|Max" $O/r05j_tests.log | head -40
exit $rc
