#!/bin/bash
# Iteration loop on the GPU box: GPU tests, then bench (+rocprof stats). && chained.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
TAG="${TAG:-iter}"
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout 300 ${PYTEST_ARGS} > gpurun_out/gpu_tests_${TAG}.log 2>&1 && \
TAG=$TAG bash scripts/gpu_bench.sh
rc=$?
echo "rc=$rc" >> gpurun_out/gpu_tests_${TAG}.log
exit $rc
