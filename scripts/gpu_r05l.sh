#!/bin/bash
# Round-5 GPU run l: Vecchia standard deviations (stochastic Fisher information) + the latent factor kernel.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_stddev_vecchia.py tests/test_gpu_optim.py tests/test_gpu_latent.py > $O/r05l_tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed|Error" $O/r05l_tests.log | head -30
exit $rc
