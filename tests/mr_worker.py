"""One rank of a multi-rank parity run (launched by tests/test_multirank.py via
torch.distributed.run; every rank drives the same GPU through the host
transport).  Rank 0 runs the CPU oracle on the same workload and prints one
`MR_RESULT {json}` line: final state, counts and step count must match the
single-rank BSP restatement bit for bit."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np                       # noqa: E402
import torch.distributed as dist         # noqa: E402

from ponyc_amd import workloads as W     # noqa: E402
from ponyc_amd.dist import GlooTransport, GlobalView   # noqa: E402
from ponyc_amd.engine import Engine      # noqa: E402

CASES = {
    "ring": (lambda e: W.ring(e, 64, 4, 100), W.ring_result, {}),
    "ring1": (lambda e: W.ring(e, 1, 3, 7), W.ring_result, {}),
    "ubench": (lambda e: W.ubench(e, 4096, 4, 32), W.ubench_result, {}),
    "ubench_det": (lambda e: W.ubench(e, 3001, 3, det=True, hops=40), W.ubench_result, {}),
    "fanin": (lambda e: W.fanin(e, 5000, 16, 20, 1), W.fanin_result, {}),
    "gups": (lambda e: W.gups(e, 14, 8, 64, 64, 3), W.gups_result, {}),
    "storm": (lambda e: W.storm(e, 3000, 4, 12), lambda e, w: e.state_read(w["type"]), {}),
    "fifo": (lambda e: W.fifo(e, 64, 7, 10, 4, batch=7, mailbox_cap=1024), W.fifo_result, {}),
    # 600 sends per source per step: sequence numbers past 511 use the high
    # bits of the 16-B cross-rank record's 14-bit seq (engine_dev.h XRec)
    "fifo_seq": (lambda e: W.fifo(e, 4, 3, 1, 600, mailbox_cap=2048), W.fifo_result, {}),
    # actors created by behaviours: every rank numbers the gathered spawn list
    "spreader": (lambda e: W.spreader(e, 10), W.spreader_result, {}),
    # backpressure across ranks: overloaded sinks mute senders on the other rank
    "mute": (lambda e: W.fifo(e, 600, 3, 3, 2, batch=10, mailbox_cap=16), W.fifo_result, {}),
    # priority sinks drain batch after batch while their senders live on both ranks
    "priority": (lambda e: W.fifo(e, 600, 3, 3, 2, batch=10, mailbox_cap=16, sink_priority=1),
                 W.fifo_result, {}),
    # zone overflow on one rank halts the next step on every rank until grown
    "spill": (lambda e: W.fifo(e, 300, 3, 4, 9, batch=4, mailbox_cap=1), W.fifo_result,
              {"mailbox_cap": 1}),
    # one sink (rank 0 only): its zone overflows on rank 0 alone, in the last
    # step of a run — run one step at a time, and run_fixed one step at a time
    "spill_one_rank": (lambda e: W.fifo(e, 300, 1, 4, 9, batch=4, mailbox_cap=1), W.fifo_result,
                       {"mailbox_cap": 1}, "steps"),
    "spill_one_rank_fixed": (lambda e: W.fifo(e, 300, 1, 4, 9, batch=4, mailbox_cap=1),
                             W.fifo_result, {"mailbox_cap": 1}, "fixed"),
    # 64 cross-rank records per peer segment against ~8K per step: the
    # exchange keeps the rest in its spill list, grows, and drops nothing
    "xspill": (lambda e: W.ubench(e, 4096, 4, 32), W.ubench_result, {"max_exchange": 64}),
    "xspill_det": (lambda e: W.ubench(e, 3001, 3, det=True, hops=40), W.ubench_result,
                   {"max_exchange": 16}, "steps"),
    # ~2048 FIFO sinks per rank taking 140 arrivals each, half of them from
    # the other rank: every rank grows its sink zone 14x in one burst (and its
    # spill lists after it), then drains 5 a step from backlogs of 135
    "backlog": (lambda e: W.fifo(e, 4095 * 140, 4095, 1, 1, batch=5, mailbox_cap=16),
                W.fifo_result, {"mailbox_cap": 16}),
    # 2*2048*638 + 1 actors: rank 0 owns 639 zones' worth of 2048 and rank 1
    # exactly 638, on either side of the 640-bucket geometry switch — both
    # ranks must still pick the same zone size (engine.hip relayout_zones)
    "zones_edge": (lambda e: W.ubench(e, 2 * 2048 * 638 + 1, 1, det=True, hops=3),
                   W.ubench_result, {}),
    # behaviours as programs (GPU_ACTOR_HT_PROGRAM): sends across ranks
    "ring_prog": (lambda e: W.ring_prog(e, 64, 4, 100), lambda e, w: e.state_read(w["type"]), {}),
    "det_prog": (lambda e: W.det_prog(e, 3001, 3, hops=40), lambda e, w: e.state_read(w["type"]), {}),
}


def drive(eng, mode: str) -> int:
    """run to quiescence: in one call, one step per call, or run_fixed(1) steps"""
    if mode == "run":
        return eng.run(0)
    steps = 0
    while True:
        if mode == "steps":
            k = eng.run(1)
        else:
            if eng.counts()["pending"] == 0:
                break
            eng.run_fixed(1)
            k = 1
        if k == 0:
            break
        steps += k
    return steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("--rccl", action="store_true",
                    help="use the RCCL exchange (needs one GPU per rank)")
    ap.add_argument("--same-gpu", action="store_true", help="every rank on device 0")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    setup, result, kw, *mode = CASES[a.case]
    mode = mode[0] if mode else "run"
    if a.rccl:
        from ponyc_amd.dist import share_comm_id
        lr = 0 if a.same_gpu else int(os.environ.get("LOCAL_RANK", rank))
        eng = Engine(device=lr, n_ranks=world, rank=rank, comm_id=share_comm_id(Engine), **kw)
    else:
        eng = Engine(device=0, n_ranks=world, rank=rank, transport=GlooTransport(), **kw)
    w = setup(eng)
    steps = drive(eng, mode)
    c = eng.counts()
    peer_write = eng.debug_info()["peer_write"]
    res = result(GlobalView(eng), w)
    eng.shutdown()
    if rank == 0:
        import pyoracle
        o = pyoracle.Oracle()
        wo = setup(o)
        so = o.run(0)
        co = o.counts()
        ro = result(o, wo)
        o.shutdown()
        out = {
            "case": a.case, "world": world,
            "state_equal": bool(np.array_equal(res, ro)),
            "steps": [int(steps), int(so)],
            "delivered": [c["delivered"], co["delivered"]],
            "sent": [c["sent"], co["sent"]],
            "pending": [c["pending"], co["pending"]],
            "by_type": c["delivered_by_type"] == co["delivered_by_type"],
            "dropped": c["dropped"], "remote": c["remote"], "peer_write": peer_write,
        }
        print("MR_RESULT " + json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
