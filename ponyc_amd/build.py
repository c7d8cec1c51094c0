"""Build libgpuactor.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m ponyc_amd.build            # the engine
    python -m ponyc_amd.build --stamps   # + libgpuactor_stamps.so, a diagnostic
                                         #   build with per-phase clock stamps

Every .hip file under csrc/ is one translation unit: engine.hip (host side,
C-ABI, helper kernels, k_sparse) and one step_*.hip per compiled k_step
instantiation. They compile in parallel into ponyc_amd/build/<variant>/ and
link into one shared library.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SRCS = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith(".hip")]
HDRS = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith(".h")] + \
       [os.path.join(ROOT, "include", "gpu_actor.h")]
OUT = os.path.join(HERE, "libgpuactor.so")
OUT_STAMPS = os.path.join(HERE, "libgpuactor_stamps.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PONYC_AMD_ARCH", "gfx950")
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
         "-Wall", "-Wno-unused-parameter", "-Wno-unused-variable"]


def _newer(out: str, deps: list[str]) -> bool:
    """out exists and is at least as new as every dep"""
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(d) <= t for d in deps)


def build(force: bool = False, verbose: bool = False, stamps: bool = False,
          defines: list[str] | None = None, out: str | None = None, jobs: int = 0) -> str:
    """Compile the translation units that are out of date (in parallel) and
    link. `defines` (-D...) and `out` make an A/B variant build."""
    defines = list(defines or []) + (["-DGPA_STAMPS"] if stamps else [])
    out = out or (OUT_STAMPS if stamps else OUT)
    variant = os.path.splitext(os.path.basename(out))[0]
    objdir = os.path.join(HERE, "build", variant)
    os.makedirs(objdir, exist_ok=True)
    stamp = os.path.join(objdir, "defines.txt")
    want = " ".join(defines)
    if not os.path.exists(stamp) or open(stamp).read() != want:
        force = True
        with open(stamp, "w") as f:
            f.write(want)
    objs, todo = [], []
    for src in SRCS:
        obj = os.path.join(objdir, os.path.basename(src)[:-4] + ".o")
        objs.append(obj)
        if force or not _newer(obj, [src] + HDRS + [stamp]):
            todo.append((src, obj))

    def compile_one(job):
        src, obj = job
        cmd = [HIPCC, *FLAGS, *defines, "-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    if todo:
        n = jobs or min(len(todo), max(1, min(8, os.cpu_count() or 1)))
        with ThreadPoolExecutor(n) as ex:
            list(ex.map(compile_one, todo))
    if todo or not _newer(out, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs, "-lrccl"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build(force=force, verbose=True))
    if "--stamps" in sys.argv:
        print(build(force=force, verbose=True, stamps=True))
