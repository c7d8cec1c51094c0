"""Phase shares of k_step's two-pass path for message-local tables (zone_dev.h
`dp`) from the diagnostic build (libgpuactor_stamps.so), C2-det workload
(1M det pingers x 5, hops 1000): median over zones of the shader-clock cycles
of count + first pass (0->1), scans + index (1->7), reserve + scan + the
actors' registers (7->8), the four rounds (8->4; drain: slot 9, tile emit:
slot 10), tail (4->6); and the real-time span of the zones (slots 11/12,
the 100 MHz clock). Only shares are meaningful (stamps perturb the kernel)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PONYC_AMD_LIB", os.path.join(ROOT, "ponyc_amd", "libgpuactor_stamps.so"))
sys.path.insert(0, ROOT)
from ponyc_amd.engine import Engine  # noqa: E402
from ponyc_amd import workloads as W  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
eng = Engine(mailbox_cap=16)
W.ubench(eng, N, 5, det=True, hops=1000)
eng.run_fixed(8)
print(f"drain_ms per step {eng.last_drain_ms():.4f}")
lib = eng.lib
lib.gpu_actor_debug_stamps.restype = ctypes.c_int
lib.gpu_actor_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
nz = eng.debug_info()["zones"]
buf = np.zeros(nz * 24, dtype=np.uint64)
lib.gpu_actor_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size)
st = buf.reshape(nz, 24).astype(np.int64)
ok = st[:, 8] > 0
print(f"zones {nz}, dp zones (stamp 8 set) {int(ok.sum())}")
st = st[ok]
tot = st[:, 6] - st[:, 0]
parts = [("count + pass 1", st[:, 1] - st[:, 0]), ("scans + index", st[:, 7] - st[:, 1]),
         ("reserve + scan", st[:, 8] - st[:, 7]), ("rounds", st[:, 4] - st[:, 8]),
         ("  drain", st[:, 9]), ("  tile emit", st[:, 10]), ("tail", st[:, 6] - st[:, 4])]
print(f"median zone span {np.median(tot):.0f} clk")
for name, v in parts:
    print(f"  {name:16s} median {np.median(v):9.0f} clk  share {np.median(v / np.maximum(tot, 1)):.3f}")
rt0, rt1 = st[:, 11], st[:, 12]
t0 = rt0.min()
print("real time (us from the first zone start): span median %.2f, end median %.2f max %.2f" % (
    np.median(rt1 - rt0) / 100.0, np.median(rt1 - t0) / 100.0, (rt1 - t0).max() / 100.0))
