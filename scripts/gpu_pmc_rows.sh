#!/bin/bash
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
# GPU box: two PMC passes (SQ counters) over the exact Vecchia bench (row kernel), each its own run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/pmc_rows
TAG="${TAG:-r02}"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_WAVES"
P3="SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_CVT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv \
      -d "$R/gpurun_out/pmc_rows/p$i" -o rows -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-latent --no-dense --no-fit --no-grouped ${PMC_BENCH_ARGS:-} \
      > "$R/gpurun_out/pmc_rows/p$i.log" 2>&1 ) || exit 1
  python scripts/pmc_by_kernel.py gpurun_out/pmc_rows/p$i gpurun_out/pmc_rows_${TAG}_p$i.txt > /dev/null || exit 1
done
