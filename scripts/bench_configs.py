"""Throughput of every BASELINE.json config on one GPU (bench.py measures C2
only, as the task contract asks; this reports the others for DESIGN.md).

Each workload is built with ponyc_amd.workloads at its BASELINE size and run
to quiescence with gpu_actor_run; rate = delivered messages / wall time of the
run (host sends done before the clock starts). One JSON line per config.
usage: python scripts/bench_configs.py [names...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ponyc_amd import workloads as W          # noqa: E402
from ponyc_amd.engine import Engine          # noqa: E402

M = 1 << 20
CONFIGS = {
    # C1: examples/ring --size 1000 --count 100 --pass 10000 (the CPU plumbing case)
    "c1_ring": (lambda e: W.ring(e, 1000, 100, 10000), {}),
    # C2, deterministic form (budgeted): 1M pingers x 5 tokens x 32 hops
    "c2_ubench_det": (lambda e: W.ubench(e, M, 5, det=True, hops=32), {}),
    # C3: fan-in, 100K senders -> 4 analyzers x 100 messages
    "c3_fanin": (lambda e: W.fanin(e, 100_000, 4, 100, 0), {}),
    # C4: gups_basic, 2^24 table over 8 updaters, 64 streamers x 1024 x 100
    "c4_gups": (lambda e: W.gups(e, 24, 8, 64, 1024, 100), {}),
    # C5, one GPU's share: 8M actors, token ring + 4 random pings each, 16 hops
    "c5_storm_8m": (lambda e: W.storm(e, 8 * M, 4, 16), {}),
}


def main():
    names = sys.argv[1:] or list(CONFIGS)
    for name in names:
        setup, kw = CONFIGS[name]
        e = Engine(**kw)
        setup(e)
        e.sync()
        t0 = time.perf_counter()
        steps = e.run()
        e.sync()
        secs = time.perf_counter() - t0
        c = e.counts()
        e.shutdown()
        print(json.dumps({"config": name, "steps": steps, "delivered": c["delivered"],
                          "seconds": round(secs, 4), "msgs_per_s": round(c["delivered"] / secs, 1),
                          "dropped": c["dropped"]}), flush=True)


if __name__ == "__main__":
    main()
