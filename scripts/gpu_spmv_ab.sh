#!/bin/bash
# GPU-box: operator (A = B^T D^-1 B + W) kernel forms at n = 100k, t = 51 and t = 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O; : > $O/spmv_ab.log
for f in ${FORMS:-"0,0,0" "0,1,2048" "0,1,1024" "16,0,0" "16,1,2048" "16,1,1024"}; do
  echo "== form $f" >> $O/spmv_ab.log
  GPBOOST_AMD_SPMV=$f GPBOOST_AMD_TIMING=1 timeout -k 10 120 python -u scripts/prof_latent_one.py ${LIK:-bernoulli_logit} 100000 80 2>&1 | grep "latent timing" >> $O/spmv_ab.log || exit $?
done
echo done >> $O/spmv_ab.log
