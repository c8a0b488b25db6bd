#!/bin/bash
# Round-5 GPU run h: VIF parity, timing at n = 100k and a kernel-trace profile.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
rm -rf $O/r05h_prof; mkdir -p $O/r05h_prof
timeout -k 10 600 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_vif.py \
  > $O/r05h_tests.log 2>&1 || { tail -30 $O/r05h_tests.log; exit 3; }
tail -2 $O/r05h_tests.log
timeout -k 10 300 python3 -u scripts/vif_probe.py > $O/r05h_probe.log 2>&1 || { cat $O/r05h_probe.log; exit 1; }
cat $O/r05h_probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05h_prof -o vif -- python3 -u scripts/vif_probe.py > $O/r05h_prof.log 2>&1 || { tail -20 $O/r05h_prof.log; exit 2; }
f=$(find $O/r05h_prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -16
