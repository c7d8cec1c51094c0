"""Phase costs of a sparse k_step (diagnostic build libgpuactor_stamps.so).

One ring of 1000 actors with one token (C1 --count 1): one message per
superstep in a one-zone world, so every phase is pure latency. Prints zone 0's
shader-clock cycles per phase (zone_dev.h GPA_STAMP) for the last step, and
the kernel's HIP-event time from run_fixed.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PONYC_AMD_LIB"] = os.path.join(ROOT, "ponyc_amd", "libgpuactor_stamps.so")
sys.path.insert(0, ROOT)
from ponyc_amd import workloads as W  # noqa: E402
from ponyc_amd.engine import Engine  # noqa: E402

eng = Engine()
W.ring(eng, 1000, 1, 1000)
eng.run_fixed(64)
lib = eng.lib
lib.gpu_actor_debug_stamps.restype = ctypes.c_int
lib.gpu_actor_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
buf = np.zeros(8, dtype=np.uint64)
lib.gpu_actor_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size)
st = buf.astype(np.int64)
names = ["count", "scans", "place S", "handlers", "reserve", "scatter"]
print(f"one-zone ring step: span {st[6] - st[0]} clk; step_ms(events)={eng.last_drain_ms():.4f}")
for i, nm in enumerate(names):
    print(f"  {nm:10s} {st[i + 1] - st[i]:9d} clk")
eng.shutdown()
