#!/bin/bash
# A/B of FITC's split-K Gram with 128- vs 64-tiles (GPBOOST_AMD_SPLITK_TILE), after the FITC tests
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fitc.py > gpurun_out/splitk_tests.log 2>&1 \
  || { tail -20 gpurun_out/splitk_tests.log; exit 1; }
tail -1 gpurun_out/splitk_tests.log
: > gpurun_out/ab_splitk.log
for rep in 1 2 3; do
  for t in 128 64; do
    GPBOOST_AMD_SPLITK_TILE=$t timeout -k 10 200 python bench.py --only-fitc --steps 10 --no-cpu-baseline > gpurun_out/ab_splitk_b.log 2>&1 || exit 2
    python -c "import json;d=json.loads(open('gpurun_out/ab_splitk_b.log').read().strip().splitlines()[-1]);d=d.get('fitc',d);print('tile $t', round(d['ms_per_step'],3), d['config']['nll'])" >> gpurun_out/ab_splitk.log
  done
done
cat gpurun_out/ab_splitk.log
