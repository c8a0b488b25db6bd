#!/bin/bash
# GPU-box round check: smoke -> GPU test suite -> bench (with CPU baseline) -> latent timing ->
# rocprofv3 kernel-trace summary of the bench. Each GPU step has its own limit; any failure
# other than test assertion failures (pytest rc 1) ends the script before the next GPU step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O/prof
TAG="${TAG:-r02}"
step() { echo "== $* $(date +%T)" >> $O/round.log; }
: > $O/round.log
step smoke
timeout -k 10 300 python -u __graft_entry__.py > $O/smoke.log 2>&1 || { echo "smoke rc=$?" >> $O/round.log; exit 1; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/round.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "$SKIP_BENCH" ] && exit $rc
step bench
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/bench_${TAG}.json 2> $O/bench_${TAG}.err || { echo "bench rc=$?" >> $O/round.log; exit 1; }
step latent
GPBOOST_AMD_TIMING=1 timeout -k 10 600 python -u scripts/time_latent.py > $O/latent_time.log 2>&1 || { echo "latent rc=$?" >> $O/round.log; exit 1; }
step rocprof
# eager launches under the profiler: its tracer does not survive hipGraph replay on this image
( cd /tmp && export TMPDIR=/tmp && GPBOOST_AMD_NO_GRAPH=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$O/prof/${TAG}" -o run -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} \
    > "$R/$O/prof_${TAG}.log" 2>&1 ) || { echo "rocprof rc=$?" >> $O/round.log; exit 1; }
find "$O/prof/${TAG}" -name "*kernel_trace.csv" -size +32M -delete
step done
exit $rc
