#!/bin/bash
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
# GPU box: HBM-side traffic of the single-vector operator kernels (scripts/prof_op1.py):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (they cannot share one pass on gfx950).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/pmc_op1t
i=0
for P in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  ( cd /tmp && export TMPDIR=/tmp GPBOOST_AMD_NO_GRAPH=1 && timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv \
      -d "$R/gpurun_out/pmc_op1t/p$i" -o op -- python3 "$R/scripts/prof_op1.py" \
      > "$R/gpurun_out/pmc_op1t/p$i.log" 2>&1 ) || { tail -5 "$R/gpurun_out/pmc_op1t/p$i.log"; exit 1; }
  python scripts/pmc_by_kernel.py gpurun_out/pmc_op1t/p$i gpurun_out/pmc_op1t_p$i.txt > /dev/null || exit 1
  rm -rf gpurun_out/pmc_op1t/p$i
done
grep -h "apply1" gpurun_out/pmc_op1t_p*.txt
