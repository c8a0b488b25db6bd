#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/latent_phase.log
timeout -k 10 300 python -m pytest tests/test_gpu_latent.py -q -x --timeout 120 -k "tight or edge" >> gpurun_out/latent_phase.log 2>&1
echo "tests rc=$?" >> gpurun_out/latent_phase.log
for n in 20000 100000; do
  echo "== n=$n" >> gpurun_out/latent_phase.log
  GPBOOST_AMD_BENCH_PRECOND=1 timeout -k 10 300 python scripts/prof_latent_one.py gaussian $n 2>&1 | grep "precond bench" >> gpurun_out/latent_phase.log
done
echo done >> gpurun_out/latent_phase.log
