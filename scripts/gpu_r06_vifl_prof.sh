#!/bin/bash
# Round 6: kernel profile of the VIF Laplace evaluation at n = 20000 (m = 200, nn = 30).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vifl_prof -o vifl -- \
  python scripts/vifl_time.py 20000 > gpurun_out/vifl_prof.log 2>&1
echo "rc=$?" >> gpurun_out/vifl_prof.log
find gpurun_out/vifl_prof -name "*kernel_stats*" | head -3
