#!/bin/bash
# GPU-box check: smoke, then the GPU test suite. Each GPU step has its own time limit;
# steps are chained with && so nothing else touches the GPU after a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 300 ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/gpu_tests.log
exit $rc
