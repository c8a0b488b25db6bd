#!/bin/bash
# full GPU suite + smoke + default bench + rocprofv3 kernel stats of a short exact bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_r01h
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01h_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/r01h_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r01h_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/r01h_bench.json 2> gpurun_out/r01h_bench.err || exit $?
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r01h" -o exact --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-latent --steps 50 > "$R/gpurun_out/prof_r01h/run.log" 2>&1
