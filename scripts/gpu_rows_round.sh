#!/bin/bash
# Row-kernel iteration on the GPU box: Vecchia parity tests (default library), then an A/B of
# library variants on the headline leg (VARIANTS, built beforehand with GPBOOST_AMD_VARIANT), then
# optionally the row-kernel PMC passes (PMC=1). Each GPU step time-limited, chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_vecchia.py tests/test_gpu_optim.py -q -x --timeout 120 --timeout-method thread \
  > gpurun_out/rows_tests.log 2>&1 || exit $?
BENCH_ARGS="--no-dense --no-fit --no-grouped" bash scripts/gpu_ab_variants.sh > /dev/null 2>&1 || exit $?
if [ "${PMC:-0}" = 1 ]; then TAG=${TAG:-r03} bash scripts/gpu_pmc_rows.sh || exit $?; fi
