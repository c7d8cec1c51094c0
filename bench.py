"""bench.py — actor msgs/sec on the gpu_actor engine (BASELINE.json metric).

Workload (BASELINE.json configs[1]): examples/message-ubench
scaled to 1,048,576 Pinger actors per GPU, 5 initial pings each, steady state
(no forward budget: every ping is forwarded to pinger rand.int(N), as the
reference's ping/send_pings do while `_go` is set). One "step" = one superstep:
every pinger drains its mailbox and forwards each ping.

Weak scaling: each rank owns 1,048,576 pingers of a global population of
N x 1,048,576 (hash-partitioned, id % N); pings cross GPUs through the RCCL
exchange. value = delivered messages over all ranks / max-over-ranks time of
the K timed steps.

Also reported:
  roofline     — the drain kernel's algorithmic HBM bytes per launch
                 (32 B per message: 16-B record written by the sender's zone and
                 read by the receiver's zone; 2*S + 2*M per active actor: state
                 read + write, S = 24 B for a pinger, and the mailbox head/tail
                 M = 8 B — SURVEY §8 d3's formula) / its average duration,
                 timed by HIP events bound to every 8th k_step dispatch of the
                 timed region (hipExtLaunchKernel, on the engine's stream);
  cpu_baseline — the reference runtime (oracle/_ref/libponyrt.so, built from
                 KittyMac/ponyc src/libponyrt) running the same pinger graph via
                 oracle/_ref/harness_ubench on this host's cores (rank 0, N=1).
Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--actors A]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PINGER_STATE_BYTES = 24        # rng x, y + count
# PMC summary (scripts/gpu_pmc.sh + scripts/pmc_traffic.py) of the current k_step build
PMC_TAG = "r01i"
REC_BYTES = 16
MAILBOX_BYTES = 8              # mailbox head/tail per active actor (SURVEY §8 d3's M)
# device atomic peak measured on MI355X by scripts/ubench_mem.hip (random u32
# atomicAdd over 1M counters; profiles/r01e_ubench_mem.txt)
ATOMIC_PEAK_GOPS = 26.3


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--actors", type=int, default=1 << 20, help="pingers per GPU")
    p.add_argument("--initial", type=int, default=5)
    p.add_argument("--mailbox-cap", type=int, default=16)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-budget", type=int, default=40,
                   help="forward budget of the bounded CPU sample")
    return p.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("PONYC_AMD_SAME_GPU"):      # rehearsal: every rank on device 0
        local = 0
    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        pg = dist
    return world, rank, local, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


def allmax(pg, v: float) -> float:
    if pg is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def allsum(pg, v: float) -> float:
    if pg is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return float(t.item())


def bcast_bytes(pg, rank: int, data: bytes | None) -> bytes:
    if pg is None:
        return data
    obj = [data]
    pg.broadcast_object_list(obj, src=0)
    return obj[0]


def cpu_baseline(args) -> dict | None:
    """Reference libponyrt on this host, bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import pyoracle
    except Exception:
        return None
    exe = pyoracle.harness_path("ubench")
    if not os.path.exists(exe):
        return None
    threads = max(1, min(16, os.cpu_count() or 1))
    sample = {"pingers": args.actors, "initial": args.initial, "budget": args.cpu_budget,
              "threads": threads, "noscale": 1}
    try:
        info, _ = pyoracle.run_harness("ubench", sample, None, timeout=300)
    except Exception as exc:       # report, never fake
        return {"value": None, "unit": "msgs/s", "cores": threads, "kind": "reference",
                "sample": f"failed: {exc!r}"}
    # also the single-thread rate (smaller budget: ~5 s at 1.9 M msgs/s)
    one = None
    try:
        info1, _ = pyoracle.run_harness("ubench", dict(sample, threads=1, budget=4), None,
                                        timeout=120)
        one = round(info1["msgs_per_sec"], 1)
    except Exception:
        one = None
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")),
                         None)
    except OSError:
        pass
    return {"value": round(info["msgs_per_sec"], 1), "unit": "msgs/s", "cores": threads,
            "value_1thread": one, "cpu_model": model,
            "kind": "reference",
            "sample": (f"harness_ubench on KittyMac/ponyc libponyrt (-O3, pthread scaling), "
                       f"{args.actors} pingers x {args.initial} initial pings, forward budget "
                       f"{args.cpu_budget} ({info['msgs']} msgs, {info['seconds']:.2f} s), "
                       f"--ponymaxthreads={threads} --ponynoblock --ponynoscale; value_1thread: "
                       f"--ponymaxthreads=1, forward budget 4")}


def main():
    args = parse()
    world, rank, local, pg = dist_setup(args)
    from ponyc_amd.engine import Engine, MSG_DTYPE

    comm = None
    if world > 1:
        comm = bcast_bytes(pg, rank, Engine.comm_id() if rank == 0 else None)
    n_total = args.actors * world
    kw = dict(device=local, n_ranks=world, rank=rank, mailbox_cap=args.mailbox_cap,
              max_actors=n_total + 1024,
              max_exchange=max(1 << 20, 2 * args.actors * args.initial // max(world, 1)))
    exchange = "none" if world == 1 else "rccl"
    try:
        eng = Engine(comm_id=comm, **kw)
        ok = 1.0
    except Exception as exc:        # RCCL unusable: say so, measure the host exchange
        if world == 1:
            raise
        print(f"rank {rank}: RCCL exchange unavailable ({exc}); using the host transport",
              file=sys.stderr)
        ok = 0.0
    if world > 1 and allmax(pg, 1.0 - ok) > 0:
        if ok:
            eng.shutdown()
        from ponyc_amd.dist import GlooTransport
        eng = Engine(transport=GlooTransport(), **kw)
        exchange = "host-staged (gloo)"
    # steady state: budget never reached
    budget = (1 << 62)
    ty = 0
    eng.type_register(ty, 3, 2)                 # HT_PINGER
    eng.type_param(ty, 0, n_total)
    eng.type_param(ty, 2, budget)
    eng.type_param(ty, 3, 5489)
    first = eng.create(ty, n_total)
    eng.type_param(ty, 1, first)
    # SyncLeader.tell_all_to_go: this rank injects the pings of the pingers it owns
    mine = np.arange(rank, n_total, world, dtype=np.uint64) + np.uint64(first)
    m = np.empty(mine.size * args.initial, dtype=MSG_DTYPE)
    for k in range(args.initial):
        sl = slice(k * mine.size, (k + 1) * mine.size)
        m["to"][sl] = mine.astype(np.uint32)
        m["behaviour"][sl] = 0
        m["arg"][sl] = 42
    eng.sendv(m)

    if args.warmup:
        eng.run_fixed(args.warmup)
    eng.sync()
    c0 = eng.counts()
    barrier(pg)
    eng.sync()
    t0 = time.perf_counter()
    eng.run_fixed(args.steps)
    eng.sync()
    t1 = time.perf_counter()
    barrier(pg)
    local_secs = t1 - t0
    drain_ms = eng.last_drain_ms()
    c1 = eng.counts()        # summed over ranks by the engine
    secs = allmax(pg, local_secs)
    delivered = c1["delivered"] - c0["delivered"]
    active = c1["active"] - c0["active"]
    atomics = c1["atomics"] - c0["atomics"]
    dropped = c1["dropped"]
    eng.shutdown()

    # roofline of the drain kernel on this rank (per launch)
    msgs_per_step = delivered / args.steps / world
    active_per_step = active / args.steps / world
    # B = sum_msgs 2R + sum_active_actors (2S + 2M)
    alg_bytes = (msgs_per_step * 2 * REC_BYTES
                 + active_per_step * (2 * PINGER_STATE_BYTES + 2 * MAILBOX_BYTES))
    achieved = alg_bytes / (drain_ms * 1e-3) / 1e9 if drain_ms > 0 else 0.0
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_k_step_%s.json" % PMC_TAG)
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if rank == 0:
        value = delivered / secs
        line = {
            "metric": "actor msgs/sec (node), message-ubench",
            "value": round(value, 1),
            "unit": "msgs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(secs / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (seeded xoroshiro128+ pingers)",
            "config": {
                "workload": f"message-ubench C2: {args.actors:,} pingers per GPU x "
                            f"{args.initial} initial pings, steady state",
                "actors_per_gpu": args.actors, "actors_total": n_total,
                "initial_pings": args.initial, "mailbox_cap": args.mailbox_cap, "batch": 100,
                "parallelism": f"actor hash partition x{world} (id % {world})",
                "exchange": exchange,
            },
            "msgs_per_step": round(delivered / args.steps, 1),
            # global atomics (chunk reservations, one per
            # (zone, destination bucket) per step; counted on device) per
            # delivered message, and their rate against the measured device peak
            "atomics": {
                "per_msg": round(atomics / max(delivered, 1), 5),
                "gops": round(atomics / world / args.steps / (drain_ms * 1e-3) / 1e9, 3)
                if drain_ms > 0 else None,
                "peak_gops": ATOMIC_PEAK_GOPS,
            },
            "dropped": dropped,
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "k_step", "kernel_ms": round(drain_ms, 4),
                "alg_bytes_per_launch": round(alg_bytes, 1),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
