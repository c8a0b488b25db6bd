#!/bin/bash
# PMC counter passes (separate rocprofv3 runs, --kernel-trace/--stats not combined with --pmc).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${TAG:-r01}"
mkdir -p "$R/gpurun_out/pmc/${TAG}"
cd /tmp && export TMPDIR=/tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM GRBM_GUI_ACTIVE" ${EXTRA_PMC}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc/${TAG}/p$i" -o run -- \
     python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > "$R/gpurun_out/pmc/${TAG}/p$i.log" 2>&1 || exit $?
done
