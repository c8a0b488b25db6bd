#!/bin/bash
# Round 6: the Newton mode-change cap (poisson / gamma) on the latent Vecchia and VIF paths + latent regressions.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mode_cap.py tests/test_gpu_latent_lik.py tests/test_gpu_latent_chol.py \
  tests/test_gpu_latent.py tests/test_gpu_vif_laplace.py -v --timeout 300 --timeout-method thread > gpurun_out/cap_t1.log 2>&1
echo "pytest rc=$?" >> gpurun_out/cap_t1.log
tail -5 gpurun_out/cap_t1.log
