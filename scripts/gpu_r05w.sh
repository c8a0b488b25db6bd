#!/bin/bash
# Round-5 GPU run w: rocprofv3 kernel-trace statistics (csv) of the headline leg (2000 timed evaluations) and of the
# whole default bench (HIP graph packet capture off), for profiles/r05/.
set -o pipefail
export TMPDIR=/tmp
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out"
mkdir -p $O
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05w_head -o head -- \
  python3 "$R/bench.py" --no-latent --no-dense --no-fit --no-grouped --no-fitc --no-row-shards --no-cpu-baseline \
  --steps 2000 > $O/r05w_head.json 2> $O/r05w_head.err ) || exit 1
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05w_all -o all -- \
  python3 "$R/bench.py" --no-cpu-baseline > $O/r05w_all.json 2> $O/r05w_all.err ) || exit 2
for f in $(find /tmp/r05w_head /tmp/r05w_all -name "*kernel_stats.csv"); do cp "$f" "$O/r05w_$(basename $(dirname $f))_$(basename $f)"; done
ls $O | grep r05w
