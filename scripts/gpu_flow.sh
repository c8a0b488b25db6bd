#!/bin/bash
# GPU-box: latent-path parity with the sync-free VADU solves, then timing of both precond forms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_latent.py -x -v --timeout 120 --timeout-method thread > $O/flow_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/flow_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
GPBOOST_AMD_TIMING=1 timeout -k 10 300 python -u scripts/time_latent.py gaussian bernoulli_logit > $O/flow_time.log 2>&1 || exit $?
GPBOOST_AMD_PRECOND=1 GPBOOST_AMD_TIMING=1 timeout -k 10 300 python -u scripts/time_latent.py gaussian > $O/level_time.log 2>&1
