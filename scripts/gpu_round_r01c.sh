#!/bin/bash
# full GPU test suite, smoke, then the default bench line (stops at the first crash / time limit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01c_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/r01c_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r01c_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r01c_bench.json 2> gpurun_out/r01c_bench.err
