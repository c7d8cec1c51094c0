"""Compile the run-time steps (csrc/jit_host.h) of the program sets the GPU
tests and the profiles run — into the library's code-object cache
(ponyc_amd/jit_cache/, beside libgpuactor.so; it travels with the tree) —
on the CPU, in parallel, so that no GPU run waits ~35 s for hiprtc per set.
A set whose cache entry exists is done at once.

    python scripts/jit_precompile.py [--lib path/to/libgpuactor.so]"""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def sets():
    from ponyc_amd import program as P
    from test_program import edge_program
    out = []
    for z12 in (False, True):
        out.append(([(0, P.ring_program())], z12))
        out.append(([(0, P.det_program(0))], z12))
        out.append(([(0, P.spreader_program(0))], z12))
    out.append(([(0, edge_program())], False))
    # any-mix engines of the tests (bit per table id): ring + FIFO source +
    # sink (test_hot_zones_past_kmaxhot), ring + spreader + fan-in sender
    # (test_spreader_after_other_types)
    for mask in ((1 << 1) | (1 << 9) | (1 << 10), (1 << 1) | (1 << 11) | (1 << 4)):
        out.append((mask, False))
    return out


def one(job):
    progs, z12, lib = job
    from ponyc_amd.engine import jit_compile, jit_compile_mix
    if isinstance(progs, int):
        jit_compile_mix(progs, z12, lib_path=lib)
        return f"mix {progs}", z12
    jit_compile(progs, z12, lib_path=lib)
    return len(progs), z12


if __name__ == "__main__":
    lib = None
    if "--lib" in sys.argv:
        lib = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
    jobs = [(p, z, lib) for p, z in sets()]
    with ProcessPoolExecutor(min(len(jobs), os.cpu_count() or 1)) as ex:
        for r in ex.map(one, jobs):
            print("compiled", r, flush=True)
