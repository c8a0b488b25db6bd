#!/bin/bash
# GPU-box: latent-path tests, then timing. Each GPU step has its own limit, chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_latent.py -q -x --timeout 300 > gpurun_out/latent_tests.log 2>&1 && \
timeout -k 10 600 python scripts/time_latent.py > gpurun_out/latent_time.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/latent_time.log
exit $rc
