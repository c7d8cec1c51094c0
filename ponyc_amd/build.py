"""Build libgpuactor.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m ponyc_amd.build            # the engine
    python -m ponyc_amd.build --stamps   # + libgpuactor_stamps.so, a diagnostic
                                         #   build with per-phase clock stamps
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "engine.hip")
DEPS = [os.path.join(HERE, "csrc", f) for f in sorted(os.listdir(os.path.join(HERE, "csrc")))
        if f.endswith((".hip", ".h"))] + [os.path.join(ROOT, "include", "gpu_actor.h")]
OUT = os.path.join(HERE, "libgpuactor.so")
OUT_STAMPS = os.path.join(HERE, "libgpuactor_stamps.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PONYC_AMD_ARCH", "gfx950")


def _fresh(out: str) -> bool:
    if not os.path.exists(out):
        return False
    t_out = os.path.getmtime(out)
    return all(os.path.getmtime(d) <= t_out for d in DEPS)


def build(force: bool = False, verbose: bool = False, stamps: bool = False) -> str:
    out = OUT_STAMPS if stamps else OUT
    if not force and _fresh(out):
        return out
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-parameter", "-Wno-unused-variable"]
    if stamps:
        cmd.append("-DGPA_STAMPS")
    cmd += ["-o", out, SRC, "-lrccl"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build(force=force, verbose=True))
    if "--stamps" in sys.argv:
        print(build(force=force, verbose=True, stamps=True))
