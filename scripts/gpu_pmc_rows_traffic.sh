#!/bin/bash
export GPBOOST_AMD_BENCH_FAST_EXIT=0   # bench.py: normal exit so the tracer writes its results
# GPU box: HBM traffic of the exact-path row kernel — FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 --pmc passes over the bench command — written as profiles-style JSON for bench.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
TAG="${TAG:-r02}"
mkdir -p gpurun_out/pmc_traffic
i=0
for P in FETCH_SIZE WRITE_SIZE TCC_HIT_sum; do
  i=$((i+1))
  EXTRA=""
  [ "$P" = TCC_HIT_sum ] && EXTRA="TCC_MISS_sum"
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $P $EXTRA --output-format csv \
      -d "$R/gpurun_out/pmc_traffic/p$i" -o rows -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-latent --no-dense --no-fit --no-grouped ${PMC_BENCH_ARGS:-} \
      > "$R/gpurun_out/pmc_traffic/p$i.log" 2>&1 ) || exit 1
  python scripts/pmc_by_kernel.py gpurun_out/pmc_traffic/p$i gpurun_out/pmc_traffic_${TAG}_p$i.txt > /dev/null || exit 1
done
python - "$TAG" <<'PY'
import json, re, sys
tag = sys.argv[1]
vals = {}
for i in (1, 2, 3):
    for line in open(f"gpurun_out/pmc_traffic_{tag}_p{i}.txt"):
        if "vecchia_rows16_kernel" in line:
            vals["dispatches"] = int(line.split()[0])
            for k, v in re.findall(r"(\w+)=([0-9.e+-]+)", line):
                vals[k] = float(v)
out = {"kernel": "vecchia_rows16_kernel<0, 2>",
       "command": "python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-latent --no-dense --no-fit --no-grouped",
       "dispatches": vals.get("dispatches"), "FETCH_SIZE_KB": vals.get("FETCH_SIZE"),
       "WRITE_SIZE_KB": vals.get("WRITE_SIZE"),
       "L2_hit_rate": vals.get("TCC_HIT_sum", 0) / max(1.0, vals.get("TCC_HIT_sum", 0) + vals.get("TCC_MISS_sum", 0)),
       "note": "per-dispatch means of separate rocprofv3 --pmc passes on MI355X; KiB units as reported (x 1024). Algorithmic "
               "input bytes per launch: coords 1.6 MB + nbr 12.0 MB + y 0.8 MB = 14.4 MB (gathers of 4-8 B per "
               "lane: the gfx950 x2 correction for 16-B streaming reads does not apply, left uncorrected). The "
               "kernel is fp64-VALU / LDS-latency bound; these bytes are not its roofline."}
json.dump(out, open(f"gpurun_out/pmc_rows_{tag}.json", "w"), indent=1)
print(out)
PY
