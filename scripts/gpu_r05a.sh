#!/bin/bash
# Round-5 first GPU run (each step time-limited, chained; a failure ends the script):
#   1. the GPU test suite; 2. bench.py --gpus 2 spawning its own ranks (host transport, one GPU);
#   3. row-shard schedule A/B (GPBOOST_AMD_ROWS16_SCHED 0/1/2); 4. processes left after a bench run.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/r05a_tests.log 2>&1 \
  || { tail -30 $O/r05a_tests.log; exit 1; }
tail -2 $O/r05a_tests.log
GPBOOST_AMD_BENCH_TRANSPORT=host timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-latent \
  > $O/r05a_n2.json 2> $O/r05a_n2.err || { tail -20 $O/r05a_n2.err; exit 2; }
python3 -c "import json;d=json.load(open('$O/r05a_n2.json'));print('n2', d['n_gpus'], d['value'], d['config']['nll'], d['config']['parallelism'])"
: > $O/r05a_sched.log
for rep in 1 2; do
  for sc in 0 1 2; do
    GPBOOST_AMD_ROWS16_SCHED=$sc timeout -k 10 300 python3 bench.py --steps 300 --warmup 10 --no-latent --no-dense --no-fit \
      --no-grouped --no-fitc --no-cpu-baseline > $O/r05a_s.json 2>> $O/r05a_sched.err || exit 3
    python3 -c "
import json;d=json.load(open('$O/r05a_s.json'));rs=d['row_shards']
print('sched', $sc, 'n1', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), *[(k, round(rs[k]['first']['kernel_ms'],4), round(rs[k]['last']['kernel_ms'],4), round(rs[k]['last']['wall_ms'],4)) for k in ('n2','n4','n8')], d['config']['nll'])" >> $O/r05a_sched.log
  done
done
cat $O/r05a_sched.log
ps -u "$(id -u)" -o pid,ppid,stat,etime,cmd > $O/r05a_ps_before.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-latent --no-dense --no-grouped --no-fitc > $O/r05a_b.json 2>&1 || exit 4
ps -u "$(id -u)" -o pid,ppid,stat,etime,cmd > $O/r05a_ps_after.txt
sleep 2
ps -u "$(id -u)" -o pid,ppid,stat,etime,cmd > $O/r05a_ps_after2.txt
cat $O/r05a_ps_after.txt
echo done
