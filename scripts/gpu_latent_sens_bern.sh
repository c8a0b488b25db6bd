#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/sens
mkdir -p $O
: > $O/bern.log
LIK=bernoulli_logit TAG=default timeout -k 10 200 python -u scripts/latent_sens.py >> $O/bern.log 2>&1 || exit $?
LIK=bernoulli_logit TAG=levels GPBOOST_AMD_DENSE_ROWS=0 GPBOOST_AMD_HEAD_ROWS=0 GPBOOST_AMD_TAIL_MERGE=1 timeout -k 10 200 python -u scripts/latent_sens.py >> $O/bern.log 2>&1 || exit $?
LIK=bernoulli_logit TAG=norelabel GPBOOST_AMD_NO_RELABEL=1 timeout -k 10 200 python -u scripts/latent_sens.py >> $O/bern.log 2>&1 || exit $?
cat $O/bern.log
