"""Step time of a hot non-commutative receiver burst against the pinger path at
the same message count (within 2x).

  fifo:   100,000 FIFO sources -> 4 FIFO sinks, one PUSH each (examples/fan-in's
          shape with order-sensitive receivers, mailbox_cap 16, batch 100).
          Step 1: the sources run and send; step 2: each sink's 25,000
          arrivals are sorted by the workgroup, 100 run, the rest carry.
  pinger: 100,000 message-ubench pingers, one ping each, steady state: every
          step delivers 100,000 messages to random pingers.
Each step is one gpu_actor_run_fixed(1); its time is the HIP-event step time
(gpu_actor_last_drain_ms). One JSON line per workload.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ponyc_amd import workloads as W      # noqa: E402
from ponyc_amd.engine import Engine      # noqa: E402


def steps(e, k):
    out = []
    for _ in range(k):
        e.run_fixed(1)
        out.append(round(e.last_drain_ms() * 1e3, 2))
    return out


for rep in range(2):
    e = Engine(mailbox_cap=16)
    W.fifo(e, 100_000, 4, 1, 1, mailbox_cap=16)
    f = steps(e, 4)
    info = e.debug_info()
    c = e.counts()
    e.shutdown()
    e = Engine(mailbox_cap=16)
    W.ubench(e, 100_000, 1, budget=1 << 40)
    p = steps(e, 4)
    e.shutdown()
    print(json.dumps({"rep": rep, "fifo_step_us": f, "fifo_delivered": c["delivered"],
                      "fifo_fixups": info["fixups"], "pinger_step_us": p,
                      "burst_vs_pinger": round(f[1] / max(p[1], 1e-9), 2)}))
