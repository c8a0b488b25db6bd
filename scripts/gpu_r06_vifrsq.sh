#!/bin/bash
# Round 6: VIF row Cholesky pivot by rsqrt + two Newton steps (multiplies) instead of sqrt + a division: VIF / VIF
# prediction / VIF-Laplace parity and the n = 100k VIF timing
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vif.py tests/test_gpu_vif_pred.py \
  tests/test_gpu_vif_laplace.py -p no:cacheprovider > gpurun_out/vrq_tests.log 2>&1 || { tail -30 gpurun_out/vrq_tests.log; exit 1; }
tail -2 gpurun_out/vrq_tests.log
timeout -k 10 200 python3 scripts/time_vif.py 100000 > gpurun_out/vrq_time.log 2>&1 || { cat gpurun_out/vrq_time.log; exit 1; }
cat gpurun_out/vrq_time.log
