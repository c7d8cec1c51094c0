"""Diagnostic: one hot zone of FIFO sinks against the oracle, step by step.
Prints, per case, the first step whose per-sink handled counts differ, with
the engine's counters and debug info at that step. Usage:
python scripts/diag_zone.py [step|whole]."""
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

CASES = [(2048 * 100, 2048, 1, 1, 1000, 16), (4100 * 100, 4100, 1, 1, 1000, 16),
         (2048 * 140, 2048, 1, 1, 5, 16)]
MODE = sys.argv[1] if len(sys.argv) > 1 else "step"
for c in CASES:
    src, sinks, b, m, batch, cap = c
    e = Engine(mailbox_cap=cap)
    o = pyoracle.Oracle()
    we = W.fifo(e, src, sinks, b, m, batch=batch, mailbox_cap=cap)
    wo = W.fifo(o, src, sinks, b, m, batch=batch, mailbox_cap=cap)
    out = {"case": c, "mode": MODE, "trace": []}
    for step in range(40 if MODE == "step" else 1):
        se = e.run(1 if MODE == "step" else 0)
        so = o.run(1 if MODE == "step" else 0)
        ce, co = e.counts(), o.counts()
        ge = np.asarray(W.fifo_result(e, we))
        go = np.asarray(W.fifo_result(o, wo))
        bad = np.nonzero((ge != go).any(axis=0))[0]
        rec = {"step": step, "ran": [se, so],
               "delivered": [ce["delivered"], co["delivered"]],
               "pending": [ce["pending"], co["pending"]],
               "bad": int(bad.size), "info": e.debug_info()}
        if bad.size:
            i = int(bad[0])
            rec["first_bad"] = i
            rec["handled"] = [int(ge[1, i]), int(go[1, i])]
            rec["handled_sum"] = [int(ge[1].sum()), int(go[1].sum())]
            rec["n_handled_zero"] = [int((ge[1] == 0).sum()), int((go[1] == 0).sum())]
        out["trace"].append(rec)
        if (se == 0 and so == 0) or bad.size:
            break
    print(json.dumps(out), flush=True)
    e.shutdown()
    o.shutdown()
