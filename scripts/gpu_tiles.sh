#!/bin/bash
# tile-blocked tail: latent parity suite, then preconditioner / evaluation timing with and without
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_latent.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tiles_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/tiles_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
MODES=4 GPBOOST_AMD_PRECOND_SPLIT=1 timeout -k 10 300 python -u scripts/head_ab.py > gpurun_out/tiles_ab.log 2>&1 || exit $?
MODES=4 GPBOOST_AMD_TAIL_TILES=0 timeout -k 10 300 python -u scripts/head_ab.py >> gpurun_out/tiles_ab.log 2>&1
