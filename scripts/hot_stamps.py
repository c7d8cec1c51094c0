"""Phase times of the hot receivers' zone in the 100K -> 4 FIFO burst step
(diagnostic build libgpuactor_stamps.so; zone_dev.h GPA_STAMP): the step in
which each sink's 25,000 arrivals are sorted by the workgroup.
  0->1 count   1->2 scans   2->3 place   3->7 big-group sort
  7->4 behaviours + carry-out   4->5 reserve   5->6 scatter + counters
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PONYC_AMD_LIB"] = os.path.join(ROOT, "ponyc_amd", "libgpuactor_stamps.so")
sys.path.insert(0, ROOT)
from ponyc_amd import workloads as W       # noqa: E402
from ponyc_amd.engine import Engine       # noqa: E402

e = Engine(mailbox_cap=16)
W.fifo(e, 100_000, 4, 1, 1, mailbox_cap=16)
lib = e.lib
lib.gpu_actor_debug_stamps.restype = ctypes.c_int
lib.gpu_actor_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
nz = (100_004 + 2047) // 2048
for step in range(4):
    e.run_fixed(1)
    buf = np.zeros(nz * 24, dtype=np.uint64)
    lib.gpu_actor_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size)
    st = buf.reshape(nz, 24).astype(np.int64)[0]
    order = [(0, 1, "count"), (1, 2, "scans"), (2, 3, "place"), (3, 7, "big sort"),
             (7, 15, "stage"), (15, 16, "behaviours"), (16, 4, "carry-out"), (4, 5, "reserve"), (5, 6, "scatter")]
    parts = {nm: int(st[b] - st[a]) for a, b, nm in order}
    allz = buf.reshape(nz, 24).astype(np.int64)
    ok = allz[:, 12] >= allz[:, 11]
    t0 = allz[ok, 11].min()
    print(f"step {step}: step_us={e.last_drain_ms() * 1e3:.1f} zone0 span={int(st[6] - st[0])} clk "
          f"real {0.01 * (st[12] - st[11]):.1f} us (start +{0.01 * (st[11] - t0):.1f}); "
          f"other zones end by {0.01 * (allz[ok, 12].max() - t0):.1f} us", parts)
e.shutdown()
