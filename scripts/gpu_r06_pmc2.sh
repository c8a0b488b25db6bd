#!/bin/bash
# Round 6: fresh PMC traffic of the headline row kernel (TAG r06) and of the latent operator / VADU kernels
# (pmc_ops), then the exact-path row-shard wall-time probe (no profiler).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
TAG=r06 PMC_BENCH_ARGS="--no-fitc --no-row-shards" bash scripts/gpu_pmc_rows_traffic.sh > gpurun_out/pmc_rows_r06.log 2>&1 || { tail -20 gpurun_out/pmc_rows_r06.log; exit 1; }
bash scripts/gpu_pmc_ops.sh > gpurun_out/pmc_ops_r06.log 2>&1 || { tail -20 gpurun_out/pmc_ops_r06.log; exit 1; }
timeout -k 10 200 python3 scripts/e1_wall.py > gpurun_out/e1_wall_r06.json 2> gpurun_out/e1_wall_r06.err || exit 1
cat gpurun_out/pmc_rows_r06.json gpurun_out/e1_wall_r06.json
