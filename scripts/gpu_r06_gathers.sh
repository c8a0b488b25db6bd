#!/bin/bash
# Round 6: selected-inverse gather with the position map in LDS: Cholesky-path parity, the factor / selinv profile
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_latent_chol.py \
  tests/test_gpu_vif_laplace.py -p no:cacheprovider > gpurun_out/gs_tests.log 2>&1 || { tail -30 gpurun_out/gs_tests.log; exit 1; }
tail -2 gpurun_out/gs_tests.log
bash scripts/gpu_r06_facprof.sh
