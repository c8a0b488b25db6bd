#!/bin/bash
# Round 6: PMC passes of the dense path (n = 20000) and the VIF path (n = 100k): HBM traffic (FETCH_SIZE,
# WRITE_SIZE in separate passes) and the SQ pass (MFMA busy cycles, LDS bank conflicts, wave-state split), per kernel.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out/pmc_r06
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
SQI="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVES"
for W in dense vif; do
  if [ "$W" = dense ]; then CMD="$R/scripts/time_dense.py 20000"; else CMD="$R/scripts/time_vif.py 100000"; fi
  i=0
  for P in FETCH_SIZE WRITE_SIZE "$SQ" "$SQI"; do
    i=$((i+1))
    ( cd /tmp && export TMPDIR=/tmp GPBOOST_AMD_NO_GRAPH=1 && timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv \
        -d "$R/gpurun_out/pmc_r06/${W}_p$i" -o k -- python3 $CMD > "$R/gpurun_out/pmc_r06/${W}_p$i.log" 2>&1 ) \
      || { tail -5 "$R/gpurun_out/pmc_r06/${W}_p$i.log"; exit 1; }
    python3 scripts/pmc_by_kernel.py gpurun_out/pmc_r06/${W}_p$i gpurun_out/pmc_r06/${W}_p$i.txt > /dev/null || exit 1
    find "gpurun_out/pmc_r06/${W}_p$i" -name "*.csv" -size +20M -delete
  done
done
head -12 gpurun_out/pmc_r06/dense_p3.txt gpurun_out/pmc_r06/vif_p3.txt gpurun_out/pmc_r06/vif_p4.txt
