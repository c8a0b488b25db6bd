#!/bin/bash
# Round-5 GPU run i: PMC counters of the VIF row kernels (n = 100k).
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
rm -rf $O/r05i_p1 $O/r05i_p2; mkdir -p $O/r05i_p1 $O/r05i_p2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/r05i_p1 -o p1 -- python3 -u scripts/vif_probe.py > $O/r05i_p1.log 2>&1 || { tail -5 $O/r05i_p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/r05i_p2 -o p2 -- python3 -u scripts/vif_probe.py > $O/r05i_p2.log 2>&1 || { tail -5 $O/r05i_p2.log; exit 2; }
ls $O/r05i_p1 $O/r05i_p2
