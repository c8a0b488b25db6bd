#!/bin/bash
# Round-5 GPU run c: FITC legs of the bench (Gaussian + bernoulli_logit Laplace) with their CPU baselines,
# and bench.py --gpus 2 (host transport) stdout check.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 bench.py --only-fitc --steps 5 > $O/r05c_fitc.json 2> $O/r05c_fitc.err || { tail -20 $O/r05c_fitc.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/r05c_fitc.json'))
for k,v in d.items(): print(k, round(v['ms_per_step'],3), v['config'].get('nll'), v['config'].get('newton_its'), (v.get('cpu_baseline') or {}).get('sample'))"
GPBOOST_AMD_BENCH_TRANSPORT=host timeout -k 10 240 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-latent \
  > $O/r05c_n2.json 2> $O/r05c_n2.err || { tail -20 $O/r05c_n2.err; exit 2; }
wc -l $O/r05c_n2.json
python3 -c "import json;d=json.load(open('$O/r05c_n2.json'));print('n2', d['n_gpus'], d['value'], d['config']['nll'])"
