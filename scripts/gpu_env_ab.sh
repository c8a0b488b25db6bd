#!/bin/bash
# GPU-box A/B: one short latent evaluation (n = 100k, CG capped) per environment setting.
# ENVS: ';'-separated list of space-separated VAR=value settings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O; LOG=$O/env_ab_${LIK:-bernoulli_logit}.log; : > $LOG
IFS=';' read -ra SETS <<< "${ENVS:-X=0}"
for e in "${SETS[@]}"; do
  echo "== $e" >> $LOG
  env $e GPBOOST_AMD_TIMING=1 timeout -k 10 120 python -u scripts/prof_latent_one.py ${LIK:-bernoulli_logit} ${N:-100000} ${ITS:-80} 2>&1 | grep "latent timing\|Error\|error" >> $LOG || exit $?
done
echo done >> $LOG
