"""Scan the gfx950 ISA of every csrc/*.hip for loads followed within three instructions by a full
`s_waitcnt vmcnt(0)` (serial memory round trips: a branch around each load, or a use right after it) and for
exec-mask branches, per kernel. Compiles each file with the build's flags and --save-temps into a temp dir.
Usage: python scripts/isa_wait_scan.py [min_loads] ; prints kernels with >= 40 % of their loads so followed."""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gpboost_amd.build import CXXFLAGS, ROCM  # noqa: E402

min_loads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
tmp = tempfile.mkdtemp(prefix="isa_scan_")
flags = [f for f in CXXFLAGS if f not in ("-fopenmp", "-Wall")]
for src in sorted(glob.glob(os.path.join(ROOT, "gpboost_amd", "csrc", "*.hip"))):
    obj = os.path.join(tmp, os.path.basename(src) + ".o")
    subprocess.run([os.path.join(ROCM, "bin", "hipcc")] + flags + ["-x", "hip", "-mllvm", "-amdgpu-mfma-vgpr-form",
                                                                     "-c", src, "-o", obj, "--save-temps"],
                   cwd=tmp, capture_output=True, check=True)
for f in sorted(glob.glob(os.path.join(tmp, "*-hip-amdgcn-amd-amdhsa-gfx950.s"))):
    lines = open(f).read().split("\n")
    cur, stats = None, {}
    for i, line in enumerate(lines):
        m = re.match(r"^(_Z[^:\s]+):", line)
        if m:
            cur = m.group(1)
            stats[cur] = [0, 0, 0]
            continue
        if cur is None:
            continue
        if "global_load" in line or "buffer_load" in line:
            stats[cur][0] += 1
            if any("s_waitcnt vmcnt(0)" in lines[j] for j in range(i + 1, min(i + 4, len(lines)))):
                stats[cur][1] += 1
        if "s_cbranch_execz" in line:
            stats[cur][2] += 1
    for k, (nl, nw, nb) in stats.items():
        if nl >= min_loads and nw >= 0.4 * nl:
            print(f"{os.path.basename(f).split('-hip-')[0]:18s} {k[:90]:90s} loads {nl:4d} load+wait0 {nw:4d} execz {nb:4d}")
