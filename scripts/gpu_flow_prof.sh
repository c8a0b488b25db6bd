#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
GPBOOST_AMD_FLOW_PROF=$O/flowprof GPBOOST_AMD_BENCH_PRECOND=1 timeout -k 10 120 python -u scripts/prof_latent_one.py gaussian ${N:-100000} 2 > $O/flow_prof.log 2>&1 && \
python scripts/flow_prof_analyze.py $O/flowprof_t1.bin $O/flowprof_t50.bin >> $O/flow_prof.log 2>&1
