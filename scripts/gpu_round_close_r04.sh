#!/bin/bash
# Round-4 closing run on the GPU box (each step time-limited and chained; a failure ends the script):
#   1. the full GPU test suite; 2. smoke(); 3. rocprofv3 kernel stats of the exact leg (the headline
#   kernel's average duration, to compare with bench.py's HIP-event figure); 4. PMC passes of the row
#   kernel (scripts/gpu_pmc_rows.sh)
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/close_tests.log 2>&1 \
  || { tail -20 gpurun_out/close_tests.log; exit 1; }
tail -2 gpurun_out/close_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/close_smoke.log 2>&1 || { cat gpurun_out/close_smoke.log; exit 2; }
cat gpurun_out/close_smoke.log
( cd /tmp && GPBOOST_AMD_BENCH_FAST_EXIT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/close_prof" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 200 --warmup 10 --no-cpu-baseline --no-latent --no-dense --no-fit \
    --no-grouped --no-fitc --no-row-shards > "$R/gpurun_out/close_prof.log" 2>&1 ) || { tail -20 gpurun_out/close_prof.log; exit 3; }
find gpurun_out/close_prof -name "*.csv" ! -name "*stats.csv" -delete
TAG=r04 PMC_BENCH_ARGS="--no-fitc" timeout -k 10 500 bash scripts/gpu_pmc_rows.sh > gpurun_out/close_pmc.log 2>&1 || { tail -20 gpurun_out/close_pmc.log; exit 4; }
find gpurun_out/pmc_rows -name "*.csv" ! -name "*stats.csv" -delete
echo done
