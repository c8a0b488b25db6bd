#!/bin/bash
# kernel-level profile of one latent evaluation (bernoulli_logit, n=100k, CG capped at 60 its);
# eager launches (GPBOOST_AMD_NO_GRAPH): rocprofv3 crashed in the graph path of mode 4 on this image
mkdir -p "$GRAFT_REPO_ROOT/gpurun_out/prof_r01c"
cd /tmp && export TMPDIR=/tmp
GPBOOST_AMD_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r01c" -o lat --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/prof_latent_one.py" bernoulli_logit 100000 60 > "$GRAFT_REPO_ROOT/gpurun_out/prof_r01c/run.log" 2>&1
