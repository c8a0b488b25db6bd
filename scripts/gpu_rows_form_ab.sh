#!/bin/bash
# Row-kernel A/B on the GPU box: Vecchia parity tests on the default build, then the headline bench
# leg alternating the bordered Gauss-Jordan form (default), the round-2 slot form
# (GPBOOST_AMD_ROWS_SLOTS=1) and library variants named in VARIANTS (built beforehand with
# GPBOOST_AMD_VARIANT=<name> GPBOOST_AMD_DEFS=...).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_vecchia.py tests/test_gpu_optim.py tests/test_gpu_covariates.py -q -x --timeout 300 --timeout-method thread > $O/rows_tests.log 2>&1 || exit $?
: > $O/rows_ab.log
for rep in 1 2 3; do
  for form in border slots ${VARIANTS:-}; do
    unset GPBOOST_AMD_ROWS_SLOTS GPBOOST_AMD_VARIANT
    case $form in
      border) ;;
      slots) export GPBOOST_AMD_ROWS_SLOTS=1 ;;
      *) export GPBOOST_AMD_VARIANT=$form ;;
    esac
    timeout -k 10 300 python -u bench.py --steps 400 --warmup 20 --no-latent --no-dense --no-fit --no-grouped --no-cpu-baseline \
      > $O/rows_b.json 2>> $O/rows_ab.err || exit $?
    python -c "import json;d=json.loads(open('$O/rows_b.json').read().strip().splitlines()[-1]);print('$form', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['config']['nll'])" >> $O/rows_ab.log
  done
done
unset GPBOOST_AMD_ROWS_SLOTS GPBOOST_AMD_VARIANT
cat $O/rows_ab.log
