#!/bin/bash
# Round-5 final check (each step time-limited and chained; a failure ends the script):
#   1. the full GPU test suite; 2. smoke(); 3. the default bench line (all legs, CPU baselines).
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/r05g_tests.log 2>&1
rc=$?
tail -4 $O/r05g_tests.log
grep -E "^FAILED" $O/r05g_tests.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r05g_smoke.log 2>&1 || { cat $O/r05g_smoke.log; exit 2; }
tail -3 $O/r05g_smoke.log
timeout -k 10 700 python3 bench.py > $O/r05g_bench.json 2> $O/r05g_bench.err || { tail -20 $O/r05g_bench.err; exit 3; }
python3 -c "
import json;d=json.load(open('$O/r05g_bench.json'))
print('headline', round(d['value'],1), round(d['ms_per_step'],4), d['roofline']['frac'])
for k in ('latent_iterative','dense','grouped','fitc','fitc_laplace','vif','fit','prediction'):
    v=d.get(k)
    if isinstance(v, dict): print(k, round(v.get('ms_per_step', 0) or 0, 3), (v.get('cpu_baseline') or {}).get('value'))
"
