#!/bin/bash
# Round 6: full-scale Vecchia predictions + the VIF likelihood tests (the row kernel gained a row offset).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_vif_pred.py tests/test_gpu_vif.py -v --timeout 300 \
  --timeout-method thread > gpurun_out/vif_t1.log 2>&1
echo "pytest rc=$?" >> gpurun_out/vif_t1.log
