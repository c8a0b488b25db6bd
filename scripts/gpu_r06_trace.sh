#!/bin/bash
# Round 6: rocprofv3 kernel statistics of (1) the headline leg alone (the bench command restricted to the exact path;
# its vecchia_rows16_kernel average is the roofline's kernel time) and (2) the full default bench, HIP's graph packet
# capture off (the configuration that traces graph replays without the profiler's crash)
set -o pipefail
export GPBOOST_AMD_BENCH_FAST_EXIT=0
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/trace_r06
mkdir -p $O
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/headline -o run --output-format csv -- \
  python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-latent --no-dense --no-fit --no-grouped --no-fitc \
  --no-row-shards > $O/headline.log 2>&1 || { tail -20 $O/headline.log; exit 1; }
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/bench -o run \
  --output-format csv -- python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 2; }
find $O -name "*.csv" ! -name "*stats.csv" -delete
f=$(find $O/headline -name "*kernel_stats.csv" | head -1); head -4 "$f" | cut -c1-200
grep -o '"ms_per_step": [0-9.]*\|"kernel_ms": [0-9.]*' $O/headline.log | head -3
