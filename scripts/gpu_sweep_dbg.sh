#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GPBOOST_AMD_SWEEP_NODMA=1 timeout -k 10 300 python -m pytest tests/test_gpu_latent.py -q -x --timeout 120 -k "tight" > gpurun_out/sweep_nodma.log 2>&1
echo "rc=$?" >> gpurun_out/sweep_nodma.log
timeout -k 10 300 python -m pytest tests/test_gpu_latent.py -q -x --timeout 120 -k "tight" > gpurun_out/sweep_dma.log 2>&1
echo "rc=$?" >> gpurun_out/sweep_dma.log
