set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_fitc.py tests/test_gpu_predict.py tests/test_gpu_latent_pred.py tests/test_gpu_optim.py tests/test_gpu_boost.py tests/test_gpu_covariates.py tests/test_gpu_latent.py > gpurun_out/diag_tests.log 2>&1; grep -E "FAILED|passed|failed" gpurun_out/diag_tests.log | tail -8
tail -1 gpurun_out/diag_tests.log
: > gpurun_out/ab_diag.log
for rep in 1 2; do
  for f in quad wave; do
    GPBOOST_AMD_DIAG_FORM=$f timeout -k 10 200 python bench.py --only-fitc --steps 10 --no-cpu-baseline > gpurun_out/ab_diag_fitc.log 2>&1 || exit 2
    python -c "import json;d=json.loads(open('gpurun_out/ab_diag_fitc.log').read().strip().splitlines()[-1]);d=d.get('fitc',d);print('fitc $f', round(d['ms_per_step'],3))" >> gpurun_out/ab_diag.log
    GPBOOST_AMD_DIAG_FORM=$f timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --no-latent --no-fit --no-grouped --no-fitc --no-row-shards > gpurun_out/ab_diag_dense.log 2>&1 || exit 3
    python -c "import json;d=json.loads(open('gpurun_out/ab_diag_dense.log').read().strip().splitlines()[-1]);print('dense $f', round(d['dense']['ms_per_step'],2), round(d['dense']['roofline']['frac'],4))" >> gpurun_out/ab_diag.log
  done
done
cat gpurun_out/ab_diag.log
