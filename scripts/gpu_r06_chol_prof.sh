#!/bin/bash
# Round 6: kernel statistics of the latent Vecchia Cholesky path at n = 100k (one construction + 2 evaluations).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/chol_prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/chol_prof -o chol -- python3 scripts/chol/time_chol.py 100000 2 > gpurun_out/chol_prof.log 2>&1
rc=$?
find gpurun_out/chol_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/chol_kernel_stats.csv \;
exit $rc
