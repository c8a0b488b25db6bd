#!/bin/bash
# Segmented B^T (t = 1) operator: latent / fit / shard GPU tests, then the single-vector operator
# timing and kernel statistics with the new form and with the lane-group form (GPBOOST_AMD_BT1_GROUPS).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O/bt1
timeout -k 10 600 python -u -m pytest tests/test_gpu_latent.py tests/test_gpu_optim.py tests/test_gpu_sharded.py -x -v \
  --timeout 200 --timeout-method thread > $O/bt1/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/bt1/tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
GPBOOST_AMD_PRECOND_SPLIT=1 timeout -k 10 300 python -u scripts/prof_op1.py > $O/bt1/op_seg.log 2>&1 || exit $?
GPBOOST_AMD_BT1_SCAN_SHFL=1 GPBOOST_AMD_PRECOND_SPLIT=1 timeout -k 10 300 python -u scripts/prof_op1.py > $O/bt1/op_shfl.log 2>&1 || exit $?
GPBOOST_AMD_BT1_GROUPS=1 GPBOOST_AMD_PRECOND_SPLIT=1 timeout -k 10 300 python -u scripts/prof_op1.py > $O/bt1/op_groups.log 2>&1 || exit $?
( cd /tmp && export TMPDIR=/tmp && GPBOOST_AMD_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$O/bt1/prof_seg" -o run -- python3 "$R/scripts/prof_op1.py" > "$R/$O/bt1/prof_seg.log" 2>&1 ) || exit $?
( cd /tmp && export TMPDIR=/tmp && GPBOOST_AMD_BT1_GROUPS=1 GPBOOST_AMD_NO_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$O/bt1/prof_groups" -o run -- python3 "$R/scripts/prof_op1.py" > "$R/$O/bt1/prof_groups.log" 2>&1 ) || exit $?
find "$O/bt1" -name "*kernel_trace.csv" -delete
exit $rc
