#!/bin/bash
# Row-kernel A/B over environment settings on the headline leg (GPU box).
#   CFGS="- GPBOOST_AMD_ROWS16=1" TAG=x TESTS=1 bash scripts/gpu_rows_env_ab.sh
# Each CFG is one space-free token of comma-separated VAR=value pairs ("-" = defaults); with TESTS=1
# the Vecchia GPU tests run under each setting first. Each GPU step time-limited; stops at a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/rows_env_ab_${TAG:-x}.log
: > "$OUT"
for cfg in ${CFGS:--}; do
  envs=()
  [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
  if [ "${TESTS:-0}" = 1 ]; then
    env "${envs[@]}" timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
      tests/test_gpu_vecchia.py tests/test_gpu_optim.py > gpurun_out/rows_env_tests.log 2>&1 || { echo "$cfg tests FAILED" >> "$OUT"; tail -40 gpurun_out/rows_env_tests.log >> "$OUT"; exit 1; }
    echo "$cfg tests: $(tail -1 gpurun_out/rows_env_tests.log)" >> "$OUT"
  fi
  for rep in 1 2; do
    env "${envs[@]}" timeout -k 10 120 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-latent --no-dense \
      --no-fit --no-grouped > gpurun_out/rows_env_b.log 2>&1 || { echo "$cfg bench FAILED" >> "$OUT"; tail -20 gpurun_out/rows_env_b.log >> "$OUT"; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/rows_env_b.log').read().strip().splitlines()[-1]);print('$cfg', round(d['value'],1), round(d['roofline']['kernel_ms'],4), d['config'].get('nll'))" >> "$OUT"
  done
done
cat "$OUT"
