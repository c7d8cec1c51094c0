"""Throughput of every BASELINE.json config on one GPU (bench.py measures C2
only, as the task contract asks; this reports the others for DESIGN.md).

Each workload is built with ponyc_amd.workloads at its BASELINE size and run
to quiescence with gpu_actor_run; rate = delivered messages / wall time of the
run (host sends done before the clock starts), from the second of two runs on
fresh engines (the first's time is reported beside it: it also loads the
kernels' code objects). One JSON line per config.
With --cpu, the reference runtime (oracle/_ref/harness_*, libponyrt built
from the reference sources) runs the same config on the host's cores
(--ponymaxthreads = every usable physical core, bench.py's host_cores rule,
--ponynoblock --ponynoscale) and its rate is reported beside the GPU's
("cpu_ref").
usage: python scripts/bench_configs.py [--cpu] [names...]
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
    # C1 as one ring (--count 1): a one-zone world, one k_step_run launch per 256 steps
    "c1_ring_one": (lambda e: W.ring(e, 1000, 1, 10000), {}),
    # C2, deterministic form (budgeted): 1M pingers x 5 tokens x 32 hops
    "c2_ubench_det": (lambda e: W.ubench(e, M, 5, det=True, hops=32), {}),
    # C3: fan-in, 100K senders -> 4 analyzers x 100 messages
    "c3_fanin": (lambda e: W.fanin(e, 100_000, 4, 100, 0), {}),
    # C4: gups_basic, 2^24 table over 8 updaters, 64 streamers x 1024 x 100
    "c4_gups": (lambda e: W.gups(e, 24, 8, 64, 1024, 100), {}),
    # C4 at GPU width (2^30-word table as 8 shards): the
    # reference's --streamers option raised from 4 to 1,048,576 (each a
    # sequential PolyRand stream; 512 zones fill the GPU), --chunk 16,
    # --iterate 8: 151M updates. Ceiling for the access pattern: random 64-bit
    # atomicXor over 2^30 words, 17.75 G/s (scripts/ubench_gups.hip)
    "c4_gups_wide": (lambda e: W.gups(e, 30, 8, 1 << 20, 16, 8), {}),
    # C4 at its stated size: 2^30-word table as 8 shards, 2^32 updates
    # (2^18 streamers x 4096 x (3 + 1)); checked in tests/test_gpu_fullsize.py
    "c4_gups_2p32": (lambda e: W.gups(e, 30, 8, 1 << 18, 4096, 3), {}),
    # the two C4 shapes with every streamer applying its own chunk (no
    # k_gups_apply: every update issued as its own atomic, none combined or
    # skipped) — the comparison ADVICE r05 asks for
    "c4_gups_own": (lambda e: W.gups(e, 24, 8, 64, 1024, 100), {}, {"PONYC_AMD_GUPS_DEFER": "0"}),
    "c4_gups_wide_own": (lambda e: W.gups(e, 30, 8, 1 << 20, 16, 8), {},
                         {"PONYC_AMD_GUPS_DEFER": "0"}),
    # C5, one GPU's share: 8M actors, token ring + 4 random pings each, 16 hops
    "c5_storm_8m": (lambda e: W.storm(e, 8 * M, 4, 16), {}),
    # C5 at its stated 1000 steps (41.9 G messages)
    "c5_storm_8m_1000": (lambda e: W.storm(e, 8 * M, 4, 1000), {}),
}


# reference harness + arguments for the configs it runs (oracle/harness/*.c)
CPU_REF = {
    "c1_ring": ("ring", {"size": 1000, "count": 100, "pass": 10000}),
    "c1_ring_one": ("ring", {"size": 1000, "count": 1, "pass": 10000}),
    "c3_fanin": ("fanin", {"senders": 100_000, "analyzers": 4, "msgs": 100, "seedmode": 0}),
    "c4_gups": ("gups", {"logtable": 24, "updaters": 8, "streamers": 64, "chunk": 1024,
                         "iterate": 100, "batched": 0}),
}


def cpu_ref(name):
    if name not in CPU_REF:
        return None
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    harness, args = CPU_REF[name]
    from bench import host_cores             # physical cores ∩ affinity ∩ cgroup quota
    threads = host_cores()["usable"]
    try:
        info, _ = pyoracle.run_harness(harness, dict(args, threads=threads, noscale=1), None,
                                       timeout=120)
    except Exception as exc:            # report, never fake
        return {"error": repr(exc)[:200]}
    return {"msgs_per_s": round(info["msgs_per_sec"], 1), "msgs": info["msgs"],
            "seconds": round(info["seconds"], 3), "threads": threads}


def main():
    args = sys.argv[1:]
    with_cpu = "--cpu" in args
    names = [a for a in args if a != "--cpu"] or [n for n in CONFIGS if not n.endswith("_1000")
                                                   and n != "c4_gups_2p32" and not n.endswith("_own")]
    for name in names:
        setup, kw, *env = CONFIGS[name]
        saved = {k: os.environ.get(k) for k in (env[0] if env else {})}
        os.environ.update(env[0] if env else {})
        # twice, on a fresh engine each time: the first run in a process also
        # loads its kernels' code objects (lazily, at their first launch)
        first = None
        for _ in range(2):
            e = Engine(**kw)
            setup(e)
            e.sync()
            t0 = time.perf_counter()
            steps = e.run()
            e.sync()
            secs = time.perf_counter() - t0
            c = e.counts()
            d = e.debug_info()
            e.shutdown()
            first = secs if first is None else first
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        line = {"config": name, "steps": steps, "delivered": c["delivered"],
                "seconds": round(secs, 4), "msgs_per_s": round(c["delivered"] / secs, 1),
                "first_run_seconds": round(first, 4),
                "dropped": c["dropped"], "env": env[0] if env else None,
                "cpu_ref": cpu_ref(name) if with_cpu else None}
        if d["gups_updates"]:
            # k_gups_apply's updates and the atomics it issued for them (the
            # rest were combined with a same-word update of their wave, or
            # were XORs of 0)
            line["gups_apply"] = {"updates": d["gups_updates"], "atomics": d["gups_atomics"]}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
