#!/bin/bash
# GPU-box: preconditioner cost alone (GPBOOST_AMD_BENCH_PRECOND) for each precond form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O; : > $O/precond_ab.log
for mode in ${MODES:-0 1}; do
  for n in ${SIZES:-20000 100000}; do
    echo "== mode=$mode n=$n" >> $O/precond_ab.log
    GPBOOST_AMD_PRECOND=$mode GPBOOST_AMD_BENCH_PRECOND=1 timeout -k 10 120 python -u scripts/prof_latent_one.py ${LIK:-gaussian} $n 2 >> $O/precond_ab.log 2>&1 || { echo "rc=$?" >> $O/precond_ab.log; exit 1; }
  done
done
