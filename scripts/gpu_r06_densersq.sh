#!/bin/bash
# Round 6: dense diagonal-block pivot by rsqrt + two Newton steps: the whole GPU suite, then the n = 20000 dense timing
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/drq_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/drq_tests.log | head -20; tail -5 gpurun_out/drq_tests.log; exit 1; }
tail -1 gpurun_out/drq_tests.log
timeout -k 10 300 python3 scripts/time_dense.py 20000 > gpurun_out/drq_time.log 2>&1 || { tail -5 gpurun_out/drq_time.log; exit 1; }
tail -4 gpurun_out/drq_time.log
