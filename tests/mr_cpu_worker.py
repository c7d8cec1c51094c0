"""CPU (gloo, world_size 2+) checks of the multi-rank host plumbing, launched by
tests/test_multirank.py: the ctypes callbacks the C library calls for its
host-staged exchange (exactly as engine.hip's exchange_host drives them: a
counts all-to-all, then a ragged byte all-to-all of 16-B records), the
counter all-reduce, and gather_state's reassembly of the id % R partition."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np                       # noqa: E402
import torch.distributed as dist         # noqa: E402

from ponyc_amd.dist import GlooTransport, gather_state   # noqa: E402
from ponyc_amd.engine import _wrap_transport             # noqa: E402

XREC = 16


class FakeEngine:
    """Local shard of one type: actor id lives on rank id % R (gpu_actor_owner)."""

    def __init__(self, rank, n, first, count, words):
        self.rank, self.n_ranks = rank, n
        self.first, self.count, self.words = {0: first}, {0: count}, {0: words}
        ids = np.arange(first, first + count)
        mine = ids[ids % n == rank]
        self._st = np.stack([mine.astype(np.uint64) * np.uint64(w + 1) for w in range(words)])

    def state_read(self, t):
        return self._st


def main():
    dist.init_process_group("gloo")
    r, R = dist.get_rank(), dist.get_world_size()
    a2a, ar = _wrap_transport(GlooTransport())
    rng = np.random.default_rng(1234)
    # every rank knows the full send matrix (seeded), so each can check its receive
    M = rng.integers(0, 50, size=(R, R))
    np.fill_diagonal(M, 0)
    M[0, R - 1] = 0                    # an empty pair
    for step in range(3):
        sc = (ctypes.c_uint64 * R)(*[int(M[r, p]) for p in range(R)])
        cb = (ctypes.c_uint64 * R)(*([8] * R))
        rc = (ctypes.c_uint64 * R)()
        assert a2a(None, ctypes.addressof(sc), cb, ctypes.addressof(rc), cb) == 0
        assert [rc[p] for p in range(R)] == [int(M[p, r]) for p in range(R)]
        # records: byte b of the record k sent r->p is (r*31 + p*7 + k + b + step) & 0xFF
        send = np.concatenate([((r * 31 + p * 7 + np.arange(M[r, p])[:, None] +
                                 np.arange(XREC)[None, :] + step) & 0xFF).astype(np.uint8).ravel()
                               for p in range(R)] + [np.zeros(0, np.uint8)])
        rbytes = [int(M[p, r]) * XREC for p in range(R)]
        recv = np.full(max(1, sum(rbytes)), 0xAA, np.uint8)
        sb = (ctypes.c_uint64 * R)(*[int(M[r, p]) * XREC for p in range(R)])
        rb = (ctypes.c_uint64 * R)(*rbytes)
        sptr = send.ctypes.data if send.size else 0
        assert a2a(None, sptr, sb, recv.ctypes.data, rb) == 0
        off = 0
        for p in range(R):
            exp = ((p * 31 + r * 7 + np.arange(M[p, r])[:, None] + np.arange(XREC)[None, :] +
                    step) & 0xFF).astype(np.uint8).ravel()
            assert np.array_equal(recv[off:off + exp.size], exp), (step, p)
            off += exp.size
        M = np.roll(M, 1, axis=1)
        np.fill_diagonal(M, 0)
    # counter all-reduce: u64 values above 2^32, summed exactly
    buf = np.array([r + 1, (1 << 40) + r, 0, 7], dtype=np.uint64)
    assert ar(None, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), buf.size) == 0
    assert buf.tolist() == [R * (R + 1) // 2, R * (1 << 40) + R * (R - 1) // 2, 0, 7 * R]
    # gather_state: global order restored from the id % R partition
    for first, count in ((0, 1000), (3, 17), (5, 1)):
        g = gather_state(FakeEngine(r, R, first, count, 3), 0)
        ids = np.arange(first, first + count, dtype=np.uint64)
        assert np.array_equal(g, np.stack([ids * np.uint64(w + 1) for w in range(3)]))
    dist.barrier()
    if r == 0:
        print("MR_CPU_OK", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
