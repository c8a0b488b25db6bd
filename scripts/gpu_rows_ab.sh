#!/bin/bash
# Row-kernel A/B on the GPU box: Vecchia parity tests, then the headline bench leg with the
# Gauss-Jordan broadcasts by LDS slots (default) and by DPP (GPBOOST_AMD_ROWS_DPP=1), alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_vecchia.py -q -x --timeout 300 --timeout-method thread > $O/rows_tests.log 2>&1 || exit $?
: > $O/rows_ab.log
for rep in 1 2 3; do
  for form in lds dpp; do
    if [ $form = dpp ]; then export GPBOOST_AMD_ROWS_DPP=1; else unset GPBOOST_AMD_ROWS_DPP; fi
    timeout -k 10 300 python -u bench.py --steps 400 --warmup 20 --no-latent --no-dense --no-fit --no-cpu-baseline \
      > $O/rows_b.json 2>> $O/rows_ab.err || exit $?
    python -c "import json;d=json.load(open('$O/rows_b.json'));print('$form', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['config']['nll'])" >> $O/rows_ab.log
  done
done
unset GPBOOST_AMD_ROWS_DPP
