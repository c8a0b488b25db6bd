#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/sweep_modes"
cd "$R" && timeout -k 10 300 python -m pytest tests/test_gpu_latent.py -q -x --timeout 120 -k "tight or edge" > gpurun_out/sweep_modes/tests.log 2>&1
echo "rc=$?" >> gpurun_out/sweep_modes/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/sweep_modes/graph" -o run --output-format csv -- python3 "$R/scripts/prof_latent_one.py" gaussian 20000 > "$R/gpurun_out/sweep_modes/graph.log" 2>&1 || exit $?
cd "$R" && timeout -k 10 600 python scripts/time_latent.py > gpurun_out/latent_time.log 2>&1
