#!/bin/bash
# GPU neighbour search: structure / parity tests, then construction time (GPU vs host search)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vecchia.py tests/test_gpu_latent.py -x -q --timeout 300 --timeout-method thread > gpurun_out/knn_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/knn_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-latent --steps 200 > gpurun_out/knn_bench.json 2> gpurun_out/knn_bench.err || exit $?
GPBOOST_AMD_HOST_KNN=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-latent --steps 50 > gpurun_out/knn_bench_host.json 2>> gpurun_out/knn_bench.err
