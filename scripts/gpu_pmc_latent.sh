#!/bin/bash
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
# GPU-box: kernel trace + PMC passes (one counter group per run) of a short latent evaluation
# (n = 100k, CG capped at 20 iterations) and of a short exact-Vecchia bench run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc; mkdir -p $O
export GPBOOST_AMD_NO_GRAPH=1
LAT="python3 scripts/prof_latent_one.py ${LIK:-bernoulli_logit} 100000 20"
BEN="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
summ() {
  python3 scripts/pmc_summarize.py $O/$1 $O/$1.csv || return 1
  f=$(find $O/$1 -name "*kernel_stats.csv")
  if [ -n "$f" ]; then cp $f $O/$1_kernel_stats.csv; fi
  rm -rf $O/$1
}
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/lat_trace -o run --output-format csv -- $LAT > $O/lat_trace.log 2>&1 || exit 11
summ lat_trace
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_BUSY_CYCLES"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/lat_$tag -o run --output-format csv -- $LAT > $O/lat_$tag.log 2>&1 || exit 12
  summ lat_$tag
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/ben_trace -o run --output-format csv -- $BEN > $O/ben_trace.log 2>&1 || exit 13
summ ben_trace
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/ben_$tag -o run --output-format csv -- $BEN > $O/ben_$tag.log 2>&1 || exit 14
  summ ben_$tag
done
echo done > $O/done.txt
