"""Phase split of k_sparse (diagnostic build, -DGPA_STAMPS): cycles per phase
summed over a run's supersteps, per step. usage:
  python -m ponyc_amd.build --stamps
  PONYC_AMD_LIB=ponyc_amd/libgpuactor_stamps.so python scripts/sparse_stamps.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ponyc_amd import workloads as W      # noqa: E402
from ponyc_amd.engine import Engine      # noqa: E402

PHASES = ["rank sort", "run check", "behaviours", "list swap"]
for name, setup in [("c1_ring", lambda e: W.ring(e, 1000, 100, 10000)),
                    ("c1_ring_one", lambda e: W.ring(e, 1000, 1, 10000)),
                    ("ring_10", lambda e: W.ring(e, 1000, 10, 10000))]:
    e = Engine()
    setup(e)
    steps = e.run()
    buf = (ctypes.c_uint64 * 8)()
    e.lib.gpu_actor_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    e.lib.gpu_actor_debug_stamps(buf, 8)
    e.shutdown()
    per = {PHASES[k]: round(buf[k] / max(steps, 1), 1) for k in range(4)}
    print(json.dumps({"config": name, "steps": steps, "cycles_per_step": per,
                      "total_per_step": round(sum(buf[k] for k in range(4)) / max(steps, 1), 1)}))
