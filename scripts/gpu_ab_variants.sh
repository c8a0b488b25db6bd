#!/bin/bash
# A/B of in-tree library variants (built beforehand with GPBOOST_AMD_VARIANT=<name>, see
# gpboost_amd/build.py) on the exact-path bench; optional GPU Vecchia tests per variant.
#   VARIANTS="base pu2 pls" TESTS=1 bash scripts/gpu_ab_variants.sh
set -eo pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ab_${TAG:-x}.log
: > "$OUT"
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then export GPBOOST_AMD_VARIANT=; else export GPBOOST_AMD_VARIANT=$v; fi
  if [ "${TESTS:-0}" = 1 ] && [ "$v" != base ]; then
    timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_vecchia.py \
      > gpurun_out/ab_tests_$v.log 2>&1
    echo "$v tests: $(tail -1 gpurun_out/ab_tests_$v.log)" >> "$OUT"
  fi
  for rep in 1 2; do
    timeout -k 10 120 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-latent ${BENCH_ARGS:-} \
      > gpurun_out/ab_b_$v.log 2>&1
    python -c "import json,sys;d=json.loads(open('gpurun_out/ab_b_$v.log').read().strip().splitlines()[-1]);print('$v', round(d['value'],1), round(d['roofline']['kernel_ms'],4))" >> "$OUT"
  done
done
cat "$OUT"
