#!/bin/bash
# GPU-box: row-kernel v3 vs v4 A/B (bench, no CPU baseline), the GPU test suite, then the
# preconditioner forms (level graphs vs single-launch sweep) at n = 100k.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O; : > $O/r01b.log
echo "== v3 $(date +%T)" >> $O/r01b.log
GPBOOST_AMD_ROWS_V3=1 timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline >> $O/r01b.log 2>&1 || { echo "v3 rc=$?" >> $O/r01b.log; exit 1; }
echo "== v4 $(date +%T)" >> $O/r01b.log
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline >> $O/r01b.log 2>&1 || { echo "v4 rc=$?" >> $O/r01b.log; exit 1; }
echo "== tests $(date +%T)" >> $O/r01b.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/gpu_tests_r01b.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/r01b.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== precond modes $(date +%T)" >> $O/r01b.log
MODES="1 2" SIZES="100000" timeout -k 10 300 bash scripts/gpu_precond_ab.sh || echo "precond rc=$?" >> $O/r01b.log
echo "== done $(date +%T)" >> $O/r01b.log
exit $rc
