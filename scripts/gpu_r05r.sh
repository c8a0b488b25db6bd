#!/bin/bash
# Round-5 GPU run r: the default bench, then which of this user's processes outlive it.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
ps -u "$(id -u)" -o pid,ppid,stat,etime,cmd > $O/r05r_ps_before.txt
timeout -k 10 600 python3 -u bench.py > $O/r05r_bench.json 2> $O/r05r_bench.err
rc=$?
sleep 3
ps -u "$(id -u)" -o pid,ppid,stat,etime,cmd > $O/r05r_ps_after.txt
cat $O/r05r_ps_after.txt
exit $rc
