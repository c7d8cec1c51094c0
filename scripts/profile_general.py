"""Per-step k_step time of the general handler path:
C2-det (message-ubench-det, 1M pingers x 5 pings, payload read and folded)
and C5 (storm, 8M actors, ring token + 4 random pings each), beside the C2
pinger — each run for a fixed number of busy supersteps (run_fixed: HIP
events around the launches, gpu_actor_last_drain_ms), so the figure is the
kernel's own, not the run loop's.

    python scripts/profile_general.py [--stamps] [pinger det storm det_prog]

--stamps loads libgpuactor_stamps.so and prints the median phase shares of
the last step (zone_dev.h GPA_STAMP: 0 count | 1 scans | 2 place | 3 hot sort
| 7 handlers+carry | 4 reserve | 5 scatter | 6).
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAMPS = "--stamps" in sys.argv
if STAMPS:
    os.environ["PONYC_AMD_LIB"] = os.path.join(ROOT, "ponyc_amd", "libgpuactor_stamps.so")
sys.path.insert(0, ROOT)
from ponyc_amd.engine import Engine  # noqa: E402
from ponyc_amd import workloads as W  # noqa: E402

M = 1 << 20
STEPS = 8
CASES = {
    # (setup, messages per busy step)
    "pinger": (lambda e: W.ubench(e, M, 5, budget=1 << 40), 5 * M),
    "det": (lambda e: W.ubench(e, M, 5, det=True, hops=1000), 5 * M),
    "storm": (lambda e: W.storm(e, 8 * M, 4, 1000), 5 * 8 * M),
    # C2-det's ping as a program (GPU_ACTOR_HT_PROGRAM, ponyc_amd.program)
    "det_prog": (lambda e: W.det_prog(e, M, 5, hops=1000), 5 * M),
}


def stamps(eng, n_actors):
    lib = eng.lib
    lib.gpu_actor_debug_stamps.restype = ctypes.c_int
    lib.gpu_actor_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    nz = (n_actors + 2047) // 2048
    buf = np.zeros(nz * 24, dtype=np.uint64)
    lib.gpu_actor_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size)
    st = buf.reshape(nz, 24).astype(np.int64)
    order = [0, 1, 2, 3, 7, 4, 5, 6]
    names = ["count", "scans", "place", "hot sort", "handlers+carry", "reserve", "scatter"]
    tot = st[:, 6] - st[:, 0]
    hnd = st[:, 4] - st[:, 7]
    start = st[:, 0] - st[:, 0].min()
    q = lambda x: [float(np.percentile(x, p)) for p in (50, 90, 99, 100)]
    out = {"zone_span_clk": float(np.median(tot)), "zone_span_p50_90_99_max": q(tot),
           "handlers_p50_90_99_max": q(hnd), "start_p50_90_99_max": q(start),
           "end_max": float((st[:, 6] - st[:, 0].min()).max())}
    for i, nm in enumerate(names):
        d = st[:, order[i + 1]] - st[:, order[i]]
        out[nm] = round(float(np.median(d / np.maximum(tot, 1))), 3)
    return out


def main():
    names = [a for a in sys.argv[1:] if not a.startswith("--")] or list(CASES)
    for name in names:
        setup, per_step = CASES[name]
        e = Engine(mailbox_cap=16)
        setup(e)
        e.run_fixed(2)                   # warm up: injection landed, zones sized
        e.run_fixed(STEPS)
        ms = e.last_drain_ms()
        c = e.counts()
        rec = {"case": name, "steps": STEPS, "kernel_ms_per_step": round(ms, 5),
               "msgs_per_step": per_step, "gmsgs_per_s": round(per_step / ms / 1e6, 2),
               "dropped": c["dropped"]}
        if STAMPS:
            rec["stamps"] = stamps(e, 8 * M if name == "storm" else M)
        e.shutdown()
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
