"""Diagnostic: one hot zone (2048 FIFO sinks) with growing bursts against the
oracle: which sizes / mailbox capacities diverge, with the engine's step,
drop and fixup counts."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle                              # noqa: E402
from ponyc_amd import workloads as W         # noqa: E402
from ponyc_amd.engine import Engine          # noqa: E402

CASES = []
for per in (20, 60, 100, 140):
    for cap in (16, 256):
        CASES.append((2048 * per, 2048, 1, 1, 1000, cap))
CASES.append((2000 * 140, 2000, 1, 1, 1000, 16))
CASES.append((1024 * 140, 1024, 1, 1, 1000, 16))
for c in CASES:
    src, sinks, b, m, batch, cap = c
    out = {"case": c}
    res = {}
    for name, mk in (("gpu", lambda: Engine(mailbox_cap=cap)), ("oracle", pyoracle.Oracle)):
        e = mk()
        w = W.fifo(e, src, sinks, b, m, batch=batch, mailbox_cap=cap)
        out[name + "_steps"] = e.run()
        cn = e.counts()
        out[name + "_delivered"] = cn["delivered"]
        out[name + "_dropped"] = cn.get("dropped")
        if name == "gpu":
            try:
                out["info"] = {k: v for k, v in e.debug_info().items() if isinstance(v, (int, float))}
            except Exception as ex:  # noqa: BLE001
                out["info"] = str(ex)
        res[name] = np.asarray(W.fifo_result(e, w)).reshape(-1, sinks)
        e.shutdown()
    bad = np.nonzero((res["gpu"] != res["oracle"]).any(axis=0))[0]
    out["bad_sinks"] = int(bad.size)
    print(json.dumps(out), flush=True)
