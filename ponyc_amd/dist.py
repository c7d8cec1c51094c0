"""Multi-rank plumbing for gpu_actor.

Two exchanges are available to an engine with n_ranks > 1:

* RCCL (production): rank 0 calls `Engine.comm_id()`, the id is broadcast
  (`share_comm_id`), every rank passes it as `comm_id=`; the per-superstep
  exchange then runs device-to-device over xGMI (`engine.hip: exchange`).
* Host transport (`GlooTransport`): the same exchange with the records staged
  through pinned host memory and the collectives done by torch.distributed on
  the gloo backend.  It exists so that the N>1 device path can be exercised by
  several processes sharing ONE GPU (the test box has one), and on hosts
  without xGMI peers.  It is not a fast path.

Actor `id` lives on rank `id % n_ranks` (`gpu_actor_owner`).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


class GlooTransport:
    """alltoallv / allreduce over an initialised torch.distributed process
    group (gloo).  Called from inside `gpu_actor_run*` on the calling thread."""

    def __init__(self, group=None):
        self.group = group
        self.world_size = dist.get_world_size(group)

    def alltoallv(self, send: np.ndarray, send_bytes: list[int], recv: np.ndarray,
                  recv_bytes: list[int]) -> None:
        # uint8 views of the pinned staging buffers: no copy on either side
        dist.all_to_all_single(torch.from_numpy(recv), torch.from_numpy(send),
                               output_split_sizes=list(recv_bytes),
                               input_split_sizes=list(send_bytes), group=self.group)

    def allreduce(self, buf: np.ndarray) -> None:
        t = torch.from_numpy(buf.view(np.int64).copy())
        dist.all_reduce(t, group=self.group)
        buf[:] = t.numpy().view(np.uint64)


def share_comm_id(engine_cls, group=None) -> bytes:
    """Rank 0 creates the RCCL unique id; everyone receives it (over gloo)."""
    buf = torch.zeros(128, dtype=torch.uint8)
    if dist.get_rank(group) == 0:
        buf = torch.frombuffer(bytearray(engine_cls.comm_id()), dtype=torch.uint8).clone()
    dist.broadcast(buf, 0, group=group)
    return bytes(buf.numpy().tobytes())


def allmax(x: float, group=None) -> float:
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def gather_state(eng, type_id: int, group=None) -> np.ndarray:
    """Collective: every rank's local field-major state of `type_id`, reassembled
    in global actor order ([words][count], index = id - first of the type)."""
    local = eng.state_read(type_id)
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, (eng.rank, local), group=group)
    first, count, n = eng.first[type_id], eng.count[type_id], eng.n_ranks
    out = np.zeros((eng.words[type_id], count), dtype=np.uint64)
    ids = np.arange(first, first + count, dtype=np.int64)
    for r, st in parts:
        mine = ids[ids % n == r] - first
        out[:, mine] = st
    return out


class GlobalView:
    """An Engine seen through `gather_state`: the workload result readers
    (ponyc_amd.workloads.*_result) then read the whole actor population."""

    def __init__(self, eng, group=None):
        self.eng, self.group = eng, group

    def state_read(self, type_id: int) -> np.ndarray:
        return gather_state(self.eng, type_id, self.group)
