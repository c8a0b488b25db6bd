#!/bin/bash
# Round-5 GPU run e: FITC (Gaussian + Laplace) after the Cholesky-factor solves; FITC bench legs.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fitc.py tests/test_gpu_fitc_laplace.py tests/test_gpu_latent_lik.py > $O/r05e_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" $O/r05e_tests.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --only-fitc --steps 5 --no-cpu-baseline > $O/r05e_fitc.json 2> $O/r05e_fitc.err || { tail -20 $O/r05e_fitc.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/r05e_fitc.json'))
for k,v in d.items(): print(k, round(v['ms_per_step'],3), v['config'].get('nll'), v['config'].get('newton_its'))"
