#!/bin/bash
# Round 6: full-scale Vecchia Laplace (FSVA, cholesky) parity on the GPU, with the Gaussian VIF and sparse Cholesky suites.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_vif_laplace.py tests/test_gpu_vif.py tests/test_gpu_vif_pred.py \
  tests/test_gpu_latent_chol.py -v --timeout 300 --timeout-method thread > gpurun_out/vifl_t1.log 2>&1
echo "pytest rc=$?" >> gpurun_out/vifl_t1.log
tail -5 gpurun_out/vifl_t1.log
