#!/bin/bash
# FITC tests (inducing points bit-exact with the reference) and the k-means means A/B: member lists
# (default) vs the all-assignment scan (GPBOOST_AMD_KMEANS_SCAN=1), FITC construction time
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fitc.py > gpurun_out/km_tests.log 2>&1 \
  || { tail -30 gpurun_out/km_tests.log; exit 1; }
tail -1 gpurun_out/km_tests.log
: > gpurun_out/ab_km.log
for rep in 1 2 3; do
  for v in list scan; do
    if [ $v = scan ]; then export GPBOOST_AMD_KMEANS_SCAN=1; else unset GPBOOST_AMD_KMEANS_SCAN; fi
    timeout -k 10 200 python bench.py --only-fitc --steps 5 --no-cpu-baseline > gpurun_out/ab_km_b.log 2>&1 || exit 2
    python -c "import json;d=json.loads(open('gpurun_out/ab_km_b.log').read().strip().splitlines()[-1]);d=d.get('fitc',d);print('$v construction_s', d['config']['construction_s'], 'nll', d['config']['nll'], 'ms', round(d['ms_per_step'],3))" >> gpurun_out/ab_km.log
  done
done
cat gpurun_out/ab_km.log
# kernel stats of the list form (one FITC construction + evaluations)
unset GPBOOST_AMD_KMEANS_SCAN
( cd /tmp && GPBOOST_AMD_BENCH_FAST_EXIT=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/km_prof" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --only-fitc --steps 5 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/km_prof.log" 2>&1 ) || exit 3
find gpurun_out/km_prof -name "*.csv" ! -name "*stats.csv" -delete
grep -i kmeans gpurun_out/km_prof/run_kernel_stats.csv | cut -d, -f1-4
