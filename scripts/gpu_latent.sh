#!/bin/bash
# GPU-box: latent-path tests, then timing. Each GPU step has its own limit. Test assertion
# failures (pytest rc 1) still allow the timing step; any other failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_latent.py -q --timeout 300 > gpurun_out/latent_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/latent_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
GPBOOST_AMD_TIMING=1 timeout -k 10 600 python scripts/time_latent.py > gpurun_out/latent_time.log 2>&1
rc2=$?
echo "rc=$rc2" >> gpurun_out/latent_time.log
[ $rc -eq 0 ] && exit $rc2
exit $rc
