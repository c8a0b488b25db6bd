#!/bin/bash
# Round-4 traces on the GPU box (every step time-limited, chained; a crash ends the script):
#   1. rocprofv3 kernel stats of the FITC leg alone (bench.py --only-fitc)
#   2. the full bench under the kernel tracer with HIP's graph packet capture off
#      (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0: the configuration that traces the latent leg's hipGraph
#      replays without the r03j / r04c SIGSEGV)
#   3. (CRASH=1) the same with packet capture on (the default) and /proc/self/maps dumped before the
#      latent leg, to symbolise the crashing frames against this image's libraries
set -o pipefail
export GPBOOST_AMD_BENCH_FAST_EXIT=0
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
T=${TAG:-x}
O=gpurun_out/trace_$T
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fitc -o run --output-format csv -- \
  python bench.py --only-fitc --steps 5 --no-cpu-baseline > $O/fitc.log 2>&1 || { tail -20 $O/fitc.log; exit 1; }
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/bench -o run \
  --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1 \
  || { tail -20 $O/bench.log; exit 2; }
find $O -name "*kernel_stats.csv" | head
# only the summaries travel back (gpurun_out is pulled only below 64 MiB)
find $O -name "*.csv" ! -name "*stats.csv" -delete
if [ -n "${CRASH:-}" ]; then
  GPBOOST_AMD_DUMP_MAPS=$O/maps.txt timeout -k 10 600 rocprofv3 --kernel-trace -d $O/crash -o run \
    --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-dense --no-fit --no-grouped \
    --no-fitc > $O/crash.log 2>&1
  echo "crash run rc=$?"
  find $O -name "*.csv" ! -name "*stats.csv" -delete
  find $O -name "core*" -delete
fi
