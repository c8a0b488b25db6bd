#!/bin/bash
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
# PMC passes (one counter group per run) of a short latent evaluation with the current operator
# kernels (gaussian vecchia_latent, n = 100k, CG capped at 20 iterations; eager launches: the
# mode-4 graph path crashed rocprofv3 on this image)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp GPBOOST_AMD_NO_GRAPH=1
O=$R/gpurun_out/pmc_r01d; mkdir -p $O
LAT="python3 $R/scripts/prof_latent_one.py gaussian 100000 20"
summ() {
  python3 $R/scripts/pmc_summarize.py $O/$1 $O/$1.csv || return 1
  rm -rf $O/$1
}
cd /tmp
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/lat_$tag -o run --output-format csv -- $LAT > $O/lat_$tag.log 2>&1 || exit 12
  summ lat_$tag
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/lat_trace -o run --output-format csv -- $LAT > $O/lat_trace.log 2>&1 || exit 11
summ lat_trace
echo done > $O/done.txt
