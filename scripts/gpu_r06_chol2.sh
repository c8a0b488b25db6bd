#!/bin/bash
# Round 6: Cholesky-path tests + the tests touched by the advisor fixes, then the kernel profile at n = 100k.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_latent_chol.py tests/test_gpu_grouped.py tests/test_gpu_internal_optim.py \
  tests/test_gpu_latent.py -x -q --timeout 400 --timeout-method thread > gpurun_out/chol_t2.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/chol_t2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
GPBOOST_AMD_TIMING=1 timeout -k 10 300 python -u scripts/chol/time_chol.py 100000 3 > gpurun_out/chol_time1.log 2>&1 || exit $?
bash scripts/gpu_r06_chol_prof.sh
