"""Backlog step times of the hot FIFO receivers (scripts/hot_receiver_bench.py's
fifo workload: 100,000 sources -> 4 sinks, 25,000 arrivals each, 100 handled
per sink per step): the burst step, then the median of the next backlog
steps, HIP events per step. For A/B runs of FIFO-only builds (no pinger).
usage: python scripts/fifo_backlog.py [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ponyc_amd import workloads as W      # noqa: E402
from ponyc_amd.engine import Engine      # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 12
e = Engine(mailbox_cap=16)
W.fifo(e, 100_000, 4, 1, 1, mailbox_cap=16)
t = []
for _ in range(k):
    e.run_fixed(1)
    t.append(round(e.last_drain_ms() * 1e3, 2))
e.shutdown()
back = sorted(t[2:])
print(json.dumps({"burst_us": t[1], "backlog_median_us": back[len(back) // 2], "steps_us": t}))
