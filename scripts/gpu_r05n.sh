#!/bin/bash
# Round-5 GPU run n: FITC + Vecchia standard deviations, the optimizer, latent and FITC suites.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_stddev_fitc.py tests/test_gpu_stddev_vecchia.py tests/test_gpu_optim.py tests/test_gpu_latent.py \
  tests/test_gpu_fitc.py > $O/r05n_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed|Error|ACTUAL|DESIRED" $O/r05n_tests.log | head -40
exit $rc
