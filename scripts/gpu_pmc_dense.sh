#!/bin/bash
# GPU box: dense-path timing (n = 20000) and one PMC pass (MFMA busy, waits) over it.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG="${TAG:-r02}"
mkdir -p gpurun_out/pmc_dense
timeout -k 10 300 python scripts/time_dense.py 2000 20000 > gpurun_out/dense_time_${TAG}.log 2>&1 || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAVES \
    --output-format csv -d "$R/gpurun_out/pmc_dense/p1" -o d -- python3 "$R/scripts/time_dense.py" 20000 \
    > "$R/gpurun_out/pmc_dense/p1.log" 2>&1 ) || { tail -5 "$R/gpurun_out/pmc_dense/p1.log"; exit 1; }
python scripts/pmc_by_kernel.py gpurun_out/pmc_dense/p1 gpurun_out/pmc_dense_${TAG}.txt > /dev/null
rm -rf gpurun_out/pmc_dense/p1
