#!/bin/bash
# Round-5 GPU run v: dense Laplace (gp_approx = none, non-Gaussian likelihoods) beside the latent-likelihood suite.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_internal_optim.py \
  > $O/r05v_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed|Error|ACTUAL|DESIRED|assert" $O/r05v_tests.log | head -40
exit $rc
