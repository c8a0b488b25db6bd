#!/bin/bash
# exact-path GPU tests + a bench line without the CPU baseline / latent leg (overhead changes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vecchia.py tests/test_capi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/exact_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/exact_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-latent --steps 200 > gpurun_out/exact_bench.json 2> gpurun_out/exact_bench.err
