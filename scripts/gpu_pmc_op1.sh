#!/bin/bash
# GPU box: PMC passes over the latent operator kernels (scripts/prof_op1.py), one run per pass.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/pmc_op1
TAG="${TAG:-r02}"
P1="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
P2="FETCH_SIZE"
P3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  ( cd /tmp && export TMPDIR=/tmp GPBOOST_AMD_NO_GRAPH=1 && timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv \
      -d "$R/gpurun_out/pmc_op1/p$i" -o op -- python3 "$R/scripts/prof_op1.py" \
      > "$R/gpurun_out/pmc_op1/p$i.log" 2>&1 ) || { tail -5 "$R/gpurun_out/pmc_op1/p$i.log"; exit 1; }
  python scripts/pmc_by_kernel.py gpurun_out/pmc_op1/p$i gpurun_out/pmc_op1_${TAG}_p$i.txt > /dev/null || exit 1
  rm -rf gpurun_out/pmc_op1/p$i
done
