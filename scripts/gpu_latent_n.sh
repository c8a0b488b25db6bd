#!/bin/bash
# latent evaluation (default tolerance) at several n, for the comparison with the reference
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O=gpurun_out/sens
mkdir -p $O
: > $O/n.log
for n in ${NS:-30000 50000 70000}; do
  TAG=n$n N=$n timeout -k 10 200 python -u scripts/latent_sens.py >> $O/n.log 2>&1 || exit $?
done
cat $O/n.log
