"""Build libgpboost_amd.so in-tree for gfx950 with hipcc (no JIT, no torch extension).

    python -m gpboost_amd.build        # or gpboost_amd.build.build()

Objects go to gpboost_amd/build/, the shared library to gpboost_amd/lib/.
A/B variants: GPBOOST_AMD_VARIANT=<name> GPBOOST_AMD_DEFS="-DFOO=1 ..." builds the same sources
with extra defines into gpboost_amd/build/ab_<name>/ and gpboost_amd/lib/ab/libgpboost_amd_<name>.so,
which gpboost_amd.basic loads when GPBOOST_AMD_VARIANT is set at run time.
The library links only the HIP runtime, RCCL and the LLVM OpenMP runtime.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
VARIANT = os.environ.get("GPBOOST_AMD_VARIANT", "")
DEFS = os.environ.get("GPBOOST_AMD_DEFS", "").split() if VARIANT else []
OBJ = os.path.join(HERE, "build", f"ab_{VARIANT}") if VARIANT else os.path.join(HERE, "build")
LIBDIR = os.path.join(HERE, "lib", "ab") if VARIANT else os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, f"libgpboost_amd_{VARIANT}.so" if VARIANT else "libgpboost_amd.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("GPBOOST_AMD_ARCH", "gfx950")

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"--offload-arch={ARCH}",
            "-fopenmp", "-Wall", "-Wno-unused-function", "-Wno-unknown-pragmas",
            f"-I{os.path.join(ROOT, 'include')}", f"-I{CSRC}", f"-I{ROCM}/include"]
LDFLAGS = ["-shared", "-fopenmp", f"--offload-arch={ARCH}", f"-L{ROCM}/lib", f"-L{ROCM}/llvm/lib",
           "-lrccl", f"-Wl,-rpath,{ROCM}/lib", f"-Wl,-rpath,{ROCM}/llvm/lib"]


def sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith((".cpp", ".hip")))


def _compile(src: str) -> str:
    obj = os.path.join(OBJ, src + ".o")
    path = os.path.join(CSRC, src)
    deps = [path] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    deps.append(os.path.join(ROOT, "include", "gpboost_amd.h"))
    deps.append(os.path.abspath(__file__))
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(p) for p in deps):
        return obj
    # MFMA accumulators in VGPRs (gfx950's unified register file): without this the compiler keeps loop-carried
    # accumulators in VGPRs and copies them to and from AGPRs around every MFMA loop iteration
    lang = ["-x", "hip", "-mllvm", "-amdgpu-mfma-vgpr-form"] if src.endswith(".hip") else []
    cmd = [os.path.join(ROCM, "bin", "hipcc")] + CXXFLAGS + DEFS + lang + ["-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip():
        sys.stderr.write(r.stderr)
    return obj


def build(verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = sources()
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [os.path.join(ROCM, "bin", "hipcc")] + objs + LDFLAGS + ["-o", LIB + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        shutil.move(LIB + ".tmp", LIB)
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build()
