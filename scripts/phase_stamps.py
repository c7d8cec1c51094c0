"""Phase shares of k_step from the diagnostic build (libgpuactor_stamps.so).

Runs the bench workload for a few steps and prints, per phase, the median over
zones of the shader-clock cycles between the stamps (zone_dev.h GPA_STAMP):
  0->1 count   1->2 scans   2->3 place into S   3->4 carry-out scan + handlers
  4->5 chunk reservation   5->6 outbox scatter + counters
Only shares are meaningful (stamps perturb the kernel).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PONYC_AMD_LIB"] = os.path.join(ROOT, "ponyc_amd", "libgpuactor_stamps.so")
sys.path.insert(0, ROOT)
from ponyc_amd.engine import Engine, MSG_DTYPE  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
eng = Engine(mailbox_cap=16)
eng.type_register(0, 3, 2)
eng.type_param(0, 0, N)
eng.type_param(0, 2, 1 << 62)
first = eng.create(0, N)
eng.type_param(0, 1, first)
m = np.empty(5 * N, dtype=MSG_DTYPE)
m["to"] = np.tile(np.arange(N, dtype=np.uint32) + first, 5)
m["behaviour"] = 0
m["arg"] = 42
eng.sendv(m)
eng.run_fixed(8)
lib = eng.lib
lib.gpu_actor_debug_stamps.restype = ctypes.c_int
lib.gpu_actor_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
nz = (N + 2047) // 2048
buf = np.zeros(nz * 24, dtype=np.uint64)
lib.gpu_actor_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size)
st = buf.reshape(nz, 24).astype(np.int64)
names = ["count", "scans", "place S", "handlers", "reserve", "scatter"]
d = np.diff(st[:, :7], axis=1)
tot = st[:, 6] - st[:, 0]
print(f"zones={nz} median zone span={np.median(tot):.0f} clk; drain_ms={eng.last_drain_ms():.4f}")
for i, nm in enumerate(names):
    print(f"  {nm:10s} median {np.median(d[:, i]):9.0f} clk  share {np.median(d[:, i] / tot):.3f}")
# launch skew: when zones start relative to the first
start = st[:, 0] - st[:, 0].min()
print(f"  zone start skew: median {np.median(start):.0f} max {start.max():.0f} clk")
eng.shutdown()
