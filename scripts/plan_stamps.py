"""Phase shares of k_step's two-pass (order-free) path from the diagnostic
build (libgpuactor_stamps.so), C2 workload: median over zones of the
shader-clock cycles of
  count (0->1)  fast check (1->7)  pass 1 (7->3)  reserve (3->5)
  pass 2 (5->4; of which scans: slot 9, handlers: slot 10, tile emit: slot 2)
  tail (4->6); slot 8: wave 0's state loads landed (pass 1)
Only shares are meaningful (stamps perturb the kernel)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PONYC_AMD_LIB", os.path.join(ROOT, "ponyc_amd", "libgpuactor_stamps.so"))
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
nz = eng.debug_info()["zones"]
buf = np.zeros(nz * 24, dtype=np.uint64)
lib.gpu_actor_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size)
st = buf.reshape(nz, 24).astype(np.int64)
tot = st[:, 6] - st[:, 0]
parts = [("count", st[:, 1] - st[:, 0]), ("fast check", st[:, 7] - st[:, 1]),
         ("  class ranks", st[:, 13] - st[:, 1]), ("  fast vote", st[:, 14] - st[:, 13]),
         ("  totals", st[:, 7] - st[:, 14]),
         ("pass 1", st[:, 3] - st[:, 7]), ("  state in", st[:, 8] - st[:, 7]),
         ("reserve", st[:, 5] - st[:, 3]),
         ("pass 2", st[:, 4] - st[:, 5]), ("  scans", st[:, 9]), ("  handlers", st[:, 10]),
         ("  tile emit", st[:, 2]), ("tail", st[:, 6] - st[:, 4])]
print(f"zones={nz} median zone span={np.median(tot):.0f} clk; drain_ms={eng.last_drain_ms():.4f}")
for nm, d in parts:
    print(f"  {nm:12s} median {np.median(d):9.0f} clk  share {np.median(d / tot):.3f}")
# zone start / end on the device's 100 MHz real-time clock (slots 11, 12;
# the shader clock above is per XCD): the grid's dispatch ramp and tail
ok = (st[:, 11] > 0) & (st[:, 12] >= st[:, 11])
if ok.any():
    t0 = st[ok, 11].min()
    us = lambda v: v * 0.01                    # 10 ns ticks
    start, end = us(st[ok, 11] - t0), us(st[ok, 12] - t0)
    span = end - start
    print(f"  real time (us from the first zone start, {ok.sum()} zones): start median "
          f"{np.median(start):.2f} p90 {np.percentile(start, 90):.2f} max {start.max():.2f}; "
          f"span median {np.median(span):.2f}; end median {np.median(end):.2f} "
          f"p90 {np.percentile(end, 90):.2f} max {end.max():.2f}")
    # by XCD (workgroups are dealt to the 8 XCDs round-robin: zone % 8)
    zid = np.nonzero(ok)[0]
    for x in range(8):
        m = (zid % 8) == x
        if m.any():
            print(f"    xcd {x}: span median {np.median(span[m]):.2f} max {span[m].max():.2f}; "
                  f"end median {np.median(end[m]):.2f} max {end[m].max():.2f}")
    sl = np.argsort(end)[-8:]
    print("    last zones:", ", ".join(f"z{zid[i]} start {start[i]:.2f} end {end[i]:.2f}" for i in sl))
eng.shutdown()
