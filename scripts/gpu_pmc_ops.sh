#!/bin/bash
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
# GPU box: HBM-side traffic (rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE, separate passes) of the
# latent operator and VADU preconditioner kernels as the bench times them (scripts/prof_op1.py ->
# GPB_BenchLatentOperators(T, 20), eager launches), for t = 1 and t = 51 columns. The raw counter
# CSVs stay under gpurun_out/pmc_ops/; scripts/pmc_ops_json.py turns them into per-application bytes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/pmc_ops
for T in 1 51; do
  for P in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp GPBOOST_AMD_NO_GRAPH=1 T_OP=$T && timeout -s KILL 150 rocprofv3 --pmc $P \
        --output-format csv -d "$R/gpurun_out/pmc_ops/raw_t${T}_$P" -o op -- python3 "$R/scripts/prof_op1.py" \
        > "$R/gpurun_out/pmc_ops/t${T}_$P.log" 2>&1 ) || { tail -5 "$R/gpurun_out/pmc_ops/t${T}_$P.log"; exit 1; }
  done
done
python3 scripts/pmc_ops_json.py gpurun_out/pmc_ops gpurun_out/pmc_ops/pmc_ops.json > /dev/null
