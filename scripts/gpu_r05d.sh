#!/bin/bash
# Round-5 GPU run d: bernoulli_probit / poisson on the Vecchia-iterative and FITC Laplace paths, plus the
# latent / FITC / prediction suites touched by the shared likelihood header.
set -o pipefail
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out
mkdir -p $O
timeout -k 10 200 python3 -u scripts/diag_fitc_lik.py > $O/r05d_diag.log 2>&1 && cat $O/r05d_diag.log && \
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_latent_lik.py tests/test_gpu_fitc_laplace.py tests/test_gpu_latent.py tests/test_gpu_predict.py \
  > $O/r05d_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" $O/r05d_tests.log | tail -30
exit $rc
