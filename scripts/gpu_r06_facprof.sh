#!/bin/bash
# Round 6: kernel trace of the Cholesky Laplace-Vecchia probe (n = 100k, 2 evaluations): phase and factor breakdown
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/facprof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o chol -- python3 scripts/chol/time_chol.py 100000 1 > $O/run.log 2>&1 || { tail -10 $O/run.log; exit 1; }
f=$(find $O -name "*kernel_trace.csv" | head -1)
python3 scripts/chol/phase_stats.py "$f" > $O/phase.txt && python3 scripts/chol/factor_stats.py "$f" > $O/factor.txt
find $O -name "*kernel_trace.csv" -delete
head -3 $O/phase.txt; cat $O/factor.txt
