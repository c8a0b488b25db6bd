#!/bin/bash
# Round 6: full GPU suite, smoke and the default bench line (the round-end sequence of the driver).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/full_tests_r06.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/full_tests_r06.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r06.log 2>&1 || exit $?
timeout -k 10 360 python -u bench.py > gpurun_out/bench_r06.json 2> gpurun_out/bench_r06.err
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench_r06.err
exit $rc
