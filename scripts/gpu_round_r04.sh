#!/bin/bash
# Round-4 GPU iteration: parity tests of the changed paths, then A/B timings of the VADU
# preconditioner plan / kernel forms (plan_ab.py per setting, GPBOOST_AMD_PRECOND_SPLIT per-part
# times) and of the row-kernel library variants (bench headline leg). Every GPU step has its own
# time limit; steps are chained so nothing else touches the GPU after a failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
OUT=gpurun_out/r04_round_${TAG:-x}.log
: > "$OUT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${TEST_FILES:-tests} \
  > gpurun_out/r04_tests_${TAG:-x}.log 2>&1
rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r04_tests_${TAG:-x}.log)" >> "$OUT"
[ $rc -ne 0 ] && { tail -30 gpurun_out/r04_tests_${TAG:-x}.log; cat "$OUT"; exit $rc; }
for cfg in ${CFGS:--}; do
  echo "== $cfg" >> "$OUT"
  envs=()
  [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
  env "${envs[@]}" GPBOOST_AMD_PRECOND_SPLIT=1 PLANS="${PLANS:-2048:14336}" LIKS="${LIKS:-gaussian}" \
      timeout -k 10 300 python -u scripts/plan_ab.py >> "$OUT" 2>&1 || { cat "$OUT"; exit 1; }
done
for v in ${VARIANTS:-}; do
  if [ "$v" = base ]; then export GPBOOST_AMD_VARIANT=; else export GPBOOST_AMD_VARIANT=$v; fi
  if [ "$v" != base ]; then
    timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_vecchia.py \
      > gpurun_out/r04_vtests_$v.log 2>&1 || { tail -20 gpurun_out/r04_vtests_$v.log; exit 1; }
    echo "$v tests: $(tail -1 gpurun_out/r04_vtests_$v.log)" >> "$OUT"
  fi
  for rep in 1 2; do
    timeout -k 10 150 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-latent --no-dense --no-fit --no-fitc \
      --no-grouped > gpurun_out/r04_b_$v.log 2>&1 || { tail -20 gpurun_out/r04_b_$v.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/r04_b_$v.log').read().strip().splitlines()[-1]);print('$v', round(d['value'],1), round(d['roofline']['kernel_ms'],4))" >> "$OUT"
  done
done
unset GPBOOST_AMD_VARIANT
if [ -n "${TRACE:-}" ]; then   # the full bench (graph replay on) under the kernel tracer, last: a crash ends the call
  export TMPDIR=/tmp
  export GPBOOST_AMD_BENCH_FAST_EXIT=0   # the tracer writes its results at normal process exit
  for kv in ${TRACE_ENV:-}; do export "$kv"; done
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_${TAG:-x} -o trace -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_trace_${TAG:-x}.log 2>&1
  echo "trace rc=$?" >> "$OUT"
fi
grep -E "^==|eval=|tail_|seg_|dense|part_|tests|^base|^[a-z0-9]+ [0-9]" "$OUT"
