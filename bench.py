"""bench.py — actor msgs/sec on the gpu_actor engine (BASELINE.json metric:
"actor msgs/sec (node), message-ubench & ring").

Headline workload (BASELINE.json configs[1]): examples/
message-ubench scaled to 1,048,576 Pinger actors per GPU, 5 initial pings
each, steady state (no forward budget: every ping is forwarded to pinger
rand.int(N), as the reference's ping/send_pings do while `_go` is set). One
"step" = one superstep: every pinger drains its mailbox and forwards each ping.

Weak scaling: each rank owns 1,048,576 pingers of a global population of
N x 1,048,576 (partitioned id % N: SURVEY §8 e1's alternative to the fmix32
hash); pings cross GPUs through the RCCL
exchange. value = delivered messages over all ranks / max-over-ranks time of
the K timed steps.

Also reported on the same line:
  roofline     — k_step's algorithmic HBM bytes per launch (SURVEY §8 d3:
                 2 x 16-B record per message + (2S + 2M) per active actor,
                 S = 24 B pinger state, M = 8 B mailbox head/tail) / its
                 average duration = two HIP events on the engine's stream
                 around the K timed launches, / K (includes the launch
                 boundaries, so it never exceeds ms_per_step); `traffic` =
                 HBM bytes per launch from the rocprofv3 --pmc passes of the
                 SAME libgpuactor.so (profiles/pmc_k_step_<tag>.json carries
                 the library's sha256; null if none matches);
  cpu_baseline — the reference runtime (oracle/_ref/libponyrt.so, built from
                 KittyMac/ponyc src/libponyrt) running the same pinger graph
                 (oracle/_ref/harness_ubench) on this host: at every usable
                 physical core (--ponymaxthreads, SURVEY §8 d4, start.c:237-241)
                 and at 1 thread; `value` is its steady state (pings handled
                 in a window after warm-up, as message-ubench's report
                 interval counts them), median of 3 runs each; `budgeted` is
                 the same graph with a forward budget run to quiescence
                 (median of 5) (rank 0, N=1);
  ring         — C1, examples/ring --size 1000 --count 100 --pass 10000 on
                 the GPU (run to quiescence, median of 3) beside the same
                 reference harness at the same core counts (BASELINE names
                 "message-ubench & ring"; N=1 only).
Ranks: `--gpus N` with N > 1 runs N rank processes, one per GPU. Under a
launcher (torch.distributed.run: WORLD_SIZE set) WORLD_SIZE must equal N;
without one, bench.py starts the N ranks itself (before any GPU call) and
exits with the worst rank's status. The exchange is RCCL; if RCCL cannot be
set up the run fails (non-zero exit) unless the host-staged exchange is asked
for with --host-transport or PONYC_AMD_SAME_GPU=1 (every rank on device 0, a
rehearsal of the N-rank path on a one-GPU box; `config.ranks_share_gpu`).
Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--actors A]
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PINGER_STATE_BYTES = 24        # rng x, y + count
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
    p.add_argument("--no-ring", action="store_true")
    p.add_argument("--cpu-budget", type=int, default=10,
                   help="forward budget per pinger of the bounded CPU sample")
    p.add_argument("--cpu-runs", type=int, default=5)
    p.add_argument("--cpu-steady-runs", type=int, default=3)
    p.add_argument("--cpu-warm-ms", type=int, default=1000)
    p.add_argument("--cpu-window-ms", type=int, default=2000)
    p.add_argument("--host-transport", action="store_true",
                   help="N > 1: exchange through pinned host memory + gloo instead of RCCL")
    return p.parse_args()


def same_gpu() -> bool:
    return os.environ.get("PONYC_AMD_SAME_GPU", "") not in ("", "0")


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """No launcher and --gpus N > 1: start N rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets
    them) and return the worst exit status. This process never touches the
    GPU. If a rank fails, the others are stopped (they would wait forever at
    the first collective)."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    worst = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0:
                worst = worst or (rc if rc > 0 else 128 - rc)
                for q in live:          # exactly the processes started above
                    q.kill()
    return worst


def dist_setup(args):
    env_world = os.environ.get("WORLD_SIZE")
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} "
                         "(launch one rank per GPU, or run without a launcher)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if same_gpu():      # rehearsal: every rank on device 0
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


def bcast_bytes(pg, rank: int, data: bytes | None) -> bytes:
    if pg is None:
        return data
    obj = [data]
    pg.broadcast_object_list(obj, src=0)
    return obj[0]


# ---- host cores -------------------------------------------------------------------------
def host_cores() -> dict:
    """Physical cores of this host, and how many of them this process may use
    (affinity mask and cgroup CPU quota). The reference caps --ponymaxthreads
    at the physical core count (start.c:237-241)."""
    phys, model = set(), None
    try:
        pid = core = None
        with open("/proc/cpuinfo") as f:
            for ln in f:
                k, _, v = ln.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name" and model is None:
                    model = v
                elif k == "physical id":
                    pid = v
                elif k == "core id":
                    core = v
                elif not k and pid is not None:
                    phys.add((pid, core))
                    pid = core = None
        if pid is not None:
            phys.add((pid, core))
    except OSError:
        pass
    n_phys = len(phys) or (os.cpu_count() or 1)
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    usable = min(n_phys, affinity, quota or affinity)
    return {"model": model, "physical": n_phys, "affinity": affinity, "cgroup_quota": quota,
            "usable": usable}


def _median_runs(pyoracle, harness: str, args: dict, runs: int, timeout: float) -> dict:
    rates, secs, msgs = [], [], None
    for _ in range(runs):
        info, _ = pyoracle.run_harness(harness, args, None, timeout=timeout)
        rates.append(info["msgs_per_sec"])
        secs.append(info["seconds"])
        msgs = info["msgs"]
    return {"value": round(statistics.median(rates), 1), "runs": [round(r, 1) for r in rates],
            "msgs": msgs, "seconds_median": round(statistics.median(secs), 4)}


def cpu_reference(args, harness: str, hargs: dict, timeout: float) -> dict | None:
    """The reference libponyrt (oracle/_ref) on this host: all usable physical
    cores and 1 thread, median of args.cpu_runs runs each."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import pyoracle
    except Exception:
        return None
    if not os.path.exists(pyoracle.harness_path(harness)):
        return None
    cores = host_cores()
    n = cores["usable"]
    try:
        allc = _median_runs(pyoracle, harness, dict(hargs, threads=n, noscale=1), args.cpu_runs,
                            timeout)
        one = _median_runs(pyoracle, harness, dict(hargs, threads=1, noscale=1), args.cpu_runs,
                           timeout)
    except Exception as exc:       # report, never fake
        return {"value": None, "unit": "msgs/s", "cores": n, "kind": "reference",
                "sample": f"failed: {exc!r}"}
    return {"value": allc["value"], "unit": "msgs/s", "cores": n, "kind": "reference",
            "value_1thread": one["value"], "runs": allc["runs"], "runs_1thread": one["runs"],
            "host": cores, "msgs_per_run": allc["msgs"],
            "seconds_median": allc["seconds_median"],
            "seconds_median_1thread": one["seconds_median"]}


def cpu_steady(args, threads: int) -> dict:
    """The reference runtime in steady state, as message-ubench measures it
    (report interval, examples/message-ubench/main.pony:86-88, 288-299): no
    forward budget; the pings handled in a window after a warm-up, ramp-down
    to quiescence excluded. Median of args.cpu_steady_runs runs."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    rates = []
    for _ in range(args.cpu_steady_runs):
        info, _ = pyoracle.run_harness("ubench", {
            "pingers": args.actors, "initial": args.initial, "threads": threads, "noscale": 1,
            "warm-ms": args.cpu_warm_ms, "window-ms": args.cpu_window_ms}, None, timeout=120)
        rates.append(info["window_msgs_per_sec"])
    return {"value": round(statistics.median(rates), 1), "runs": [round(r, 1) for r in rates]}


def cpu_baseline(args) -> dict | None:
    r = cpu_reference(args, "ubench", {"pingers": args.actors, "initial": args.initial,
                                       "budget": args.cpu_budget}, timeout=300)
    if not r or r.get("value") is None:
        return r
    budgeted = {"value": r.pop("value"), "value_1thread": r.pop("value_1thread"),
                "runs": r.pop("runs"), "runs_1thread": r.pop("runs_1thread"),
                "msgs_per_run": r.pop("msgs_per_run"),
                "seconds_median": r.pop("seconds_median"),
                "seconds_median_1thread": r.pop("seconds_median_1thread"),
                "sample": (f"{args.actors} pingers x {args.initial} initial pings, forward "
                           f"budget {args.cpu_budget} per pinger, run to quiescence (ramp-down "
                           f"included); median of {args.cpu_runs} runs each; time = pony_start "
                           f"region (CLOCK_MONOTONIC)")}
    try:
        allc = cpu_steady(args, r["cores"])
        one = cpu_steady(args, 1)
    except Exception as exc:         # report, never fake
        r.update(value=None, sample=f"steady-state run failed: {exc!r}", budgeted=budgeted)
        return r
    r.update(value=allc["value"], value_1thread=one["value"], runs=allc["runs"],
             runs_1thread=one["runs"], budgeted=budgeted)
    r["sample"] = (f"harness_ubench on KittyMac/ponyc libponyrt (-O3, pthread scaling), steady "
                   f"state: {args.actors} pingers x {args.initial} initial pings, no forward "
                   f"budget; pings handled in a {args.cpu_window_ms} ms window after "
                   f"{args.cpu_warm_ms} ms of warm-up (the reference's report interval, "
                   f"message-ubench/main.pony:86-88, 288-299), then the pingers stop forwarding; "
                   f"--ponymaxthreads={r['cores']} (every usable physical core) and =1, "
                   f"--ponynoblock --ponynoscale; median of {args.cpu_steady_runs} runs each. "
                   f"`budgeted`: the same graph with a forward budget, run to quiescence")
    return r


# ---- the roofline's traffic field: PMC summary of this exact library ---------------------
def lib_sha16(path: str) -> str | None:
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


BENCH_WORKLOAD = "c2_message_ubench"


def pmc_workload(path: str, d: dict) -> str:
    """The workload a PMC summary was collected on: its `workload` field, or
    (older summaries) the tag's suffix — pmc_k_step_<tag>_det / _storm are the
    general-path passes of scripts/gpu_evidence.sh, not this bench's."""
    if d.get("workload"):
        return d["workload"]
    stem = os.path.basename(path)[: -len(".json")]
    for suffix in ("_det", "_storm"):
        if stem.endswith(suffix):
            return suffix[1:]
    return BENCH_WORKLOAD


def pmc_traffic(sha: str | None) -> tuple[float | None, str | None]:
    if sha is None:
        return None, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_k_step_*.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if (d.get("lib_sha16") == sha and d.get("hbm_bytes_per_launch")
                and pmc_workload(f, d) == BENCH_WORKLOAD):
            return d["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


# ---- C1 ring on the GPU ----------------------------------------------------------------------
def ring_gpu(reps: int = 3) -> dict:
    from ponyc_amd import workloads as W
    from ponyc_amd.engine import Engine
    out = []
    for _ in range(reps):
        e = Engine(device=0)
        W.ring(e, 1000, 100, 10000)
        e.sync()
        t0 = time.perf_counter()
        steps = e.run()
        e.sync()
        secs = time.perf_counter() - t0
        c = e.counts()
        e.shutdown()
        out.append((c["delivered"] / secs, secs, steps, c["delivered"], c["dropped"]))
    out.sort()
    v, secs, steps, delivered, dropped = out[len(out) // 2]
    return {"value": round(v, 1), "unit": "msgs/s", "seconds": round(secs, 5), "steps": steps,
            "ms_per_step": round(secs / steps * 1e3, 5), "delivered": delivered,
            "dropped": dropped, "runs": [round(o[0], 1) for o in out]}


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world, rank, local, pg = dist_setup(args)
    from ponyc_amd.engine import Engine, MSG_DTYPE, LIB_PATH

    host_xp = world > 1 and (args.host_transport or same_gpu())
    n_total = args.actors * world
    kw = dict(device=local, n_ranks=world, rank=rank, mailbox_cap=args.mailbox_cap,
              max_actors=n_total + 1024,
              max_exchange=max(1 << 20, 2 * args.actors * args.initial // max(world, 1)))
    if world == 1:
        eng = Engine(**kw)
        exchange = "none"
    elif host_xp:
        from ponyc_amd.dist import GlooTransport
        eng = Engine(transport=GlooTransport(), **kw)
        exchange = "host-staged"
    else:
        import torch
        ndev = torch.cuda.device_count()      # counts devices without initialising HIP
        if ndev < world:
            raise SystemExit(f"bench.py: {world} ranks need {world} GPUs, this node has {ndev} "
                             "(PONYC_AMD_SAME_GPU=1 rehearses N ranks on one GPU)")
        comm = bcast_bytes(pg, rank, Engine.comm_id() if rank == 0 else None)
        try:
            eng = Engine(comm_id=comm, **kw)
        except Exception as exc:
            # never measure something else silently: the rank exits non-zero
            # and the launcher (or launch_ranks) stops the others
            print(f"bench.py rank {rank}: RCCL exchange unavailable: {exc}", file=sys.stderr)
            raise SystemExit(3)
        exchange = "rccl"
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
    step_ms = eng.last_drain_ms()      # events around the K launches, / K
    c1 = eng.counts()        # summed over ranks by the engine
    secs = allmax(pg, local_secs)
    delivered = c1["delivered"] - c0["delivered"]
    active = c1["active"] - c0["active"]
    atomics = c1["atomics"] - c0["atomics"]
    dropped = c1["dropped"]
    eng.shutdown()

    # roofline of the step kernel on this rank (per launch)
    msgs_per_step = delivered / args.steps / world
    active_per_step = active / args.steps / world
    # B = sum_msgs 2R + sum_active_actors (2S + 2M)
    alg_bytes = (msgs_per_step * 2 * REC_BYTES
                 + active_per_step * (2 * PINGER_STATE_BYTES + 2 * MAILBOX_BYTES))
    achieved = alg_bytes / (step_ms * 1e-3) / 1e9 if step_ms > 0 else 0.0
    sha = lib_sha16(LIB_PATH)
    traffic, traffic_src = pmc_traffic(sha)

    cpu = ring = None
    if rank == 0 and world == 1:
        if not args.no_ring:
            ring = {"workload": "C1 examples/ring --size 1000 --count 100 --pass 10000 "
                                "(100,000 actors, 1,000,100 pass + 100 set messages), run to "
                                "quiescence",
                    **ring_gpu()}
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(args)
            if ring is not None:
                rc = cpu_reference(args, "ring", {"size": 1000, "count": 100, "pass": 10000},
                                   timeout=120)
                if rc and rc.get("value") is not None:
                    rc["sample"] = (f"harness_ring on KittyMac/ponyc libponyrt, same config, "
                                    f"--ponymaxthreads={rc['cores']} and =1, median of "
                                    f"{args.cpu_runs} runs each")
                ring["cpu_baseline"] = rc

    if rank == 0:
        value = delivered / secs
        line = {
            "metric": "actor msgs/sec (node), message-ubench & ring",
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
                # SURVEY §8 e1's alternative partition (the north star's fmix32
                # hash is not implemented): actor id -> rank id % N, local slot id / N
                "parallelism": f"actor partition id % {world} over {world} rank(s)",
                "exchange": exchange,
                "ranks_share_gpu": bool(world > 1 and same_gpu()),
            },
            "msgs_per_step": round(delivered / args.steps, 1),
            # global atomics (chunk reservations, one per
            # (zone, destination bucket) per step; counted on device) per
            # delivered message, and their rate against the measured device peak
            "atomics": {
                "per_msg": round(atomics / max(delivered, 1), 5),
                "gops": round(atomics / world / args.steps / (step_ms * 1e-3) / 1e9, 3)
                if step_ms > 0 else None,
                "peak_gops": ATOMIC_PEAK_GOPS,
            },
            "dropped": dropped,
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                # a two-pass table's step is two launches (zone_dev.h k_step PM
                # 1 and 2); the events span both
                "kernel": ("k_step<PINGER,0>" if os.environ.get("PONYC_AMD_SPLIT_PLAN") == "0"
                           else "k_step<PINGER,1> + k_step<PINGER,2>" if os.environ.get("PONYC_AMD_FUSE") == "0"
                           else "k_step<PINGER,3> (one launch: the two-pass path, the rest through a call)"),
                "kernel_ms": round(step_ms, 5),
                "kernel_ms_source": "HIP events around the timed launches on the engine stream, / steps",
                "alg_bytes_per_launch": round(alg_bytes, 1),
                "lib_sha16": sha,
            },
            "cpu_baseline": cpu,
            "ring": ring,
        }
        print(json.dumps(line))
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
