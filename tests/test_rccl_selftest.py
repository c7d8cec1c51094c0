"""The RCCL bodies of the engine's cross-rank collectives, executed.

Two ranks cannot share one GPU under RCCL ("Duplicate GPU detected"), so the
two-rank parity cases (tests/test_multirank.py) run the exchange's control
flow through the host transport, and only the nccl* calls inside the four
collectives (engine.hip xc_allreduce_sum / xc_alltoall_u64 / xc_allgather_u64
/ xc_sendrecv) are left to a multi-GPU node. This test runs each of those
RCCL bodies once on a one-rank communicator (gpu_actor_debug_rccl_selftest:
ncclCommInitAll over the engine's device), on device buffers in the engine's
stream: ncclAllReduce for u64/u32/u8, ncclAllToAll, ncclAllGather, and a
grouped ncclSend/ncclRecv. One rank sums to itself, so every output equals
its input."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_collectives_on_one_rank(engine_factory):
    e = engine_factory()
    fn = e.lib.gpu_actor_debug_rccl_selftest
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    fn.restype = ctypes.c_int
    out = np.zeros(23, dtype=np.uint64)
    rc = fn(out.ctypes.data_as(ctypes.c_void_p), out.size)
    assert rc == 0, f"gpu_actor_debug_rccl_selftest returned {rc}"
    u64 = np.array([0x1000000000 * (i + 1) + i for i in range(4)], dtype=np.uint64)
    u32 = np.array([0x10000 * (i + 1) + 7 for i in range(4)] + [0] * 4,
                   dtype=np.uint32)
    u8 = np.array([(3 * i + 1) & 0xFF for i in range(64)], dtype=np.uint8)
    np.testing.assert_array_equal(out[0:4], u64)
    np.testing.assert_array_equal(out[4:8].view(np.uint32), u32)
    np.testing.assert_array_equal(out[8:16].view(np.uint8), u8)
    assert int(out[16]) == 0xA2A0000000000001
    assert int(out[17]) == 0xA770000000000002
    np.testing.assert_array_equal(out[18:22], np.uint64(0x5E4D000000000000) + np.arange(4, dtype=np.uint64))
    assert int(out[22]) > 0                  # ncclGetVersion
    print(f"RCCL version code {int(out[22])}")
