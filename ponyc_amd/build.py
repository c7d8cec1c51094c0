"""Build libgpuactor.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m ponyc_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "engine.hip")
DEPS = [SRC, os.path.join(HERE, "csrc", "engine_dev.h"), os.path.join(HERE, "csrc", "rng_dev.h"),
        os.path.join(HERE, "csrc", "zone_dev.h"),
        os.path.join(ROOT, "include", "gpu_actor.h")]
OUT = os.path.join(HERE, "libgpuactor.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PONYC_AMD_ARCH", "gfx950")


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and os.path.exists(OUT):
        t_out = os.path.getmtime(OUT)
        if all(os.path.getmtime(d) <= t_out for d in DEPS):
            return OUT
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-parameter", "-Wno-unused-variable",
           "-o", OUT, SRC, "-lrccl"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
