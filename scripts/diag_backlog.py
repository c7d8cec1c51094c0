"""Diagnostic: FIFO backlog cases against the oracle, reporting which sinks
differ (by zone of 2048). Usage: python scripts/diag_backlog.py  (engine lib
from PONYC_AMD_LIB, PONYC_AMD_DEFER_BIG as set)."""
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

CASES = [(574_000, 4100, 1, 1, 5), (4100 * 100, 4100, 1, 1, 1000), (2048 * 140, 2048, 1, 1, 5),
         (33 * 140, 33, 1, 1, 5), (300 * 140, 300, 1, 1, 5), (4100 * 20, 4100, 1, 1, 5)]
for c in CASES:
    src, sinks, b, m, batch = c
    out = {"case": c}
    for name, mk in (("gpu", lambda: Engine(mailbox_cap=16)), ("oracle", pyoracle.Oracle)):
        e = mk()
        w = W.fifo(e, src, sinks, b, m, batch=batch, mailbox_cap=16)
        out[name + "_steps"] = e.run()
        out[name + "_delivered"] = e.counts()["delivered"]
        out[name] = np.asarray(W.fifo_result(e, w)).reshape(-1, sinks)
        e.shutdown()
    g, o = out.pop("gpu"), out.pop("oracle")
    bad = np.nonzero((g != o).any(axis=0))[0]
    out["bad_sinks"] = int(bad.size)
    out["bad_by_zone"] = np.bincount(bad // 2048, minlength=3).tolist() if bad.size else []
    out["first_bad"] = bad[:10].tolist()
    print(json.dumps(out), flush=True)
