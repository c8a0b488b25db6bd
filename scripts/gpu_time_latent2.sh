#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GPBOOST_AMD_TIMING=1 timeout -k 10 600 python scripts/time_latent.py > gpurun_out/latent_time.log 2>&1
echo "rc=$?" >> gpurun_out/latent_time.log
