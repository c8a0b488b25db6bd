#!/bin/bash
# Round-5 GPU run b: FITC-Laplace parity, bench.py --gpus 2 (own ranks, host transport), row-shard
# schedule A/B. Each step time-limited and chained.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fitc_laplace.py tests/test_gpu_fitc.py tests/test_gpu_predict.py tests/test_gpu_grouped.py -k "fitc or saved" > $O/r05b_tests.log 2>&1 \
  || { tail -40 $O/r05b_tests.log; exit 1; }
tail -3 $O/r05b_tests.log
echo "n2 bench start"
GPBOOST_AMD_BENCH_TRANSPORT=host timeout -k 10 240 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-latent \
  > $O/r05b_n2.json 2> $O/r05b_n2.err || { tail -20 $O/r05b_n2.err; exit 2; }
python3 -c "import json;d=json.load(open('$O/r05b_n2.json'));print('n2', d['n_gpus'], d['value'], d['config']['nll'], d['config']['parallelism'])"
: > $O/r05b_sched.log
for rep in 1 2; do
  for sc in 0 1 2; do
    GPBOOST_AMD_ROWS16_SCHED=$sc timeout -k 10 200 python3 bench.py --steps 300 --warmup 10 --no-latent --no-dense --no-fit \
      --no-grouped --no-fitc --no-cpu-baseline > $O/r05b_s.json 2>> $O/r05b_sched.err || exit 3
    python3 -c "
import json;d=json.load(open('$O/r05b_s.json'));rs=d['row_shards']
print('sched', $sc, 'n1', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), *[(k, round(rs[k]['first']['kernel_ms'],4), round(rs[k]['last']['kernel_ms'],4), round(rs[k]['last']['wall_ms'],4)) for k in ('n2','n4','n8')], d['config']['nll'])" | tee -a $O/r05b_sched.log
  done
done
echo done
