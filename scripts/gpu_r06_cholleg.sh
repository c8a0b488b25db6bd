#!/bin/bash
# Round 6: Cholesky Laplace-Vecchia bench leg alone (n = 100k bernoulli_logit) with the device-side breakdown
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
GPBOOST_AMD_TIMING=1 timeout -k 10 300 python3 scripts/chol/time_chol.py 100000 3 > gpurun_out/cholleg_time.log 2>&1 || { tail -20 gpurun_out/cholleg_time.log; exit 1; }
tail -12 gpurun_out/cholleg_time.log | cut -c1-200
timeout -k 10 300 python3 scripts/chol/bench_leg.py 3 --no-cpu > gpurun_out/cholleg.json 2> gpurun_out/cholleg.err || { tail -20 gpurun_out/cholleg.err; exit 1; }
cut -c1-400 gpurun_out/cholleg.json
