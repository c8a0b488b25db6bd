#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GPBOOST_AMD_SWEEP_MODE=4 timeout -k 10 300 python scripts/prof_latent_one.py gaussian 20000 > gpurun_out/sweep_prof.log 2>&1
