#!/bin/bash
# GPU-box: latent GPU tests, then latent eval timing with / without the locality relabelling.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O; : > $O/relabel.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_latent.py -x -v --timeout 200 --timeout-method thread > $O/latent_tests.log 2>&1
rc=$?; echo "latent tests rc=$rc" >> $O/relabel.log
[ $rc -eq 0 ] || exit $rc
echo "== relabel" >> $O/relabel.log
SIZES=100000 GPBOOST_AMD_TIMING=1 timeout -k 10 200 python -u scripts/time_latent.py gaussian bernoulli_logit >> $O/relabel.log 2>&1 || exit $?
echo "== no relabel" >> $O/relabel.log
GPBOOST_AMD_NO_RELABEL=1 SIZES=100000 GPBOOST_AMD_TIMING=1 timeout -k 10 200 python -u scripts/time_latent.py gaussian bernoulli_logit >> $O/relabel.log 2>&1 || exit $?
echo done >> $O/relabel.log
