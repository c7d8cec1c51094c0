"""Phase times of k_hot (hot_dev.h HOT_RT, diagnostic build
libgpuactor_stamps.so) on the hot-receiver burst: 100,000 FIFO sources -> 4
sinks; workgroup 0's real-time stamps of the burst step's k_hot launch."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PONYC_AMD_LIB", os.path.join(ROOT, "ponyc_amd", "libgpuactor_stamps.so"))
sys.path.insert(0, ROOT)
from ponyc_amd import workloads as W      # noqa: E402
from ponyc_amd.engine import Engine      # noqa: E402

e = Engine(mailbox_cap=16)
W.fifo(e, 100_000, 4, 1, 1, mailbox_cap=16)
e.run_fixed(1)
e.run_fixed(1)
print(f"burst step {e.last_drain_ms() * 1e3:.1f} us")
lib = e.lib
lib.gpu_actor_debug_stamps.restype = ctypes.c_int
lib.gpu_actor_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
buf = np.zeros(4096 * 24, dtype=np.uint64)
lib.gpu_actor_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size)
st = buf.reshape(4096, 24)[4095].astype(np.int64)
names = ["P1 count", "barrier 1", "P2 bins", "barrier 2", "P2.5 starts", "barrier 3", "P3 place",
         "barrier 4", "P4 sort", "barrier 5"]
for k, nm in enumerate(names):
    print(f"  {nm:12s} {(st[k + 1] - st[k]) * 0.01:8.2f} us")
print(f"  total        {(st[10] - st[0]) * 0.01:8.2f} us")
e.shutdown()
