#!/bin/bash
# Round-5 GPU run f: FITC after the transposed-factor solves; A/B of G = M^-1 K (factor form vs explicit inverse)
# in precision (diag script) and time (bench FITC legs).
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fitc.py tests/test_gpu_fitc_laplace.py tests/test_gpu_latent_lik.py > $O/r05f_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" $O/r05f_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
for g in inv; do
  GPBOOST_AMD_FITC_G=$g timeout -k 10 200 python3 -u scripts/diag_fitc_lik.py > $O/r05f_diag_$g.log 2>&1 || exit 3
  echo "== $g"; grep -o "rel [-0-9.e]*" $O/r05f_diag_$g.log | tr '\n' ' '; echo
  GPBOOST_AMD_FITC_G=$g timeout -k 10 300 python3 bench.py --only-fitc --steps 10 --no-cpu-baseline > $O/r05f_fitc_$g.json 2> $O/r05f_fitc_$g.err || { tail -20 $O/r05f_fitc_$g.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/r05f_fitc_$g.json'))
for k,v in d.items(): print(k, round(v['ms_per_step'],3), v['config'].get('nll'), v['config'].get('newton_its'))"
done
