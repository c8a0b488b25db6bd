#!/bin/bash
# Round-5 run s (CPU work on the GPU box's host): one measured reference dense evaluation at n = 20000 on
# 16 host threads (progress every 30 s), for bench.py's dense cpu_baseline.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 1150 python3 -u scripts/ref_dense_n20000.py 20000 16
