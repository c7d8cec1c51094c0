"""Edge cases of the boundary on the GPU (the reference's own tests pin the
same corners of the runtime: nothing to run, zero-length sends, bad ids —
pony_sendv to a non-actor is impossible in Pony, so the C-ABI rejects it).
Every case goes through libgpuactor.so; state is compared with the oracle."""
import numpy as np
import pytest

from ponyc_amd import workloads as W
from ponyc_amd.engine import MSG_DTYPE, RING_PASS, RING_SET, GpuActorError

pytestmark = pytest.mark.gpu

EINVAL, ESTATE, EBUSY = -1, -6, -9


def test_no_actors(engine_factory):
    e = engine_factory()
    assert e.run() == 0
    e.run_fixed(3)
    c = e.counts()
    assert c["delivered"] == 0 and c["sent"] == 0 and c["pending"] == 0


def test_actors_without_mail_are_quiescent(engine_factory, oracle):
    """Constructors only: no step runs and the constructed state equals the
    oracle's (ring: next / id words, examples/ring/main.pony:3-24)."""
    e = engine_factory()
    e.type_register(0, 4, W.HT_RING)
    e.type_param(0, 0, 10)
    e.create(0, 30)
    assert e.run() == 0
    oracle.type_register(0, 4, W.HT_RING)
    oracle.type_param(0, 0, 10)
    oracle.create(0, 30)
    assert oracle.run() == 0
    np.testing.assert_array_equal(e.state_read(0), oracle.state_read(0))
    e.run_fixed(2)                        # empty supersteps change nothing
    np.testing.assert_array_equal(e.state_read(0), oracle.state_read(0))
    assert e.counts()["delivered"] == 0


def test_empty_sendv_is_a_noop(engine_factory, oracle):
    g = engine_factory()
    w = W.ubench(g, 256, 2, det=True, hops=5)
    g.sendv(np.zeros(0, dtype=MSG_DTYPE))
    steps = g.run()
    wo = W.ubench(oracle, 256, 2, det=True, hops=5)
    assert steps == oracle.run()
    np.testing.assert_array_equal(W.ubench_result(g, w), W.ubench_result(oracle, wo))


def test_bad_arguments_are_rejected(engine_factory):
    e = engine_factory()
    with pytest.raises(GpuActorError) as ex:
        e.type_register(16, 1, W.HT_RING)             # >= GPU_ACTOR_MAX_TYPES
    assert ex.value.code == EINVAL
    e.type_register(0, 4, W.HT_RING)
    e.type_param(0, 0, 3)
    first = e.create(0, 3)
    with pytest.raises(GpuActorError) as ex:
        e.send(first + 3, 0, 1)                       # past the last id
    assert ex.value.code == EINVAL
    with pytest.raises(GpuActorError) as ex:
        e.send(first, 16, 1)                          # behaviour outside the table
    assert ex.value.code == EINVAL
    with pytest.raises(GpuActorError):
        e.create(0, 3)                                # a type is created once
    with pytest.raises(GpuActorError) as ex:
        e.state_read(0, 0, 4)                         # past the type's actors
    assert ex.value.code == EINVAL
    # the engine is still usable after rejected calls
    e.send(first, RING_SET, first + 1)
    e.send(first, RING_PASS, 4)
    assert e.run() > 0
    assert e.counts()["dropped"] == 0


def test_reinit_after_shutdown_repeats_bit_for_bit(engine_factory):
    """The runtime is per process: shutdown + init again gives the same run."""
    out = []
    for _ in range(2):
        e = engine_factory()
        w = W.fanin(e, 300, 3, 7, 1)
        steps = e.run()
        out.append((steps, W.fanin_result(e, w).copy(), e.counts()["delivered"]))
        e.shutdown()
    assert out[0][0] == out[1][0] and out[0][2] == out[1][2]
    np.testing.assert_array_equal(out[0][1], out[1][1])


def test_run_async_busy_and_serialised(engine_factory, oracle):
    """While an async run is in flight gpu_actor_run returns EBUSY; other calls
    wait behind it; wait() joins it."""
    e = engine_factory()
    w = W.ubench(e, 4096, 4, det=True, hops=64)
    e.run_async(0)
    try:
        e.run()                           # EBUSY unless the async run already ended
    except GpuActorError as ex:
        assert ex.code == EBUSY
    c = e.counts()                        # serialised behind the async run
    steps = e.wait()
    wo = W.ubench(oracle, 4096, 4, det=True, hops=64)
    assert steps == oracle.run()
    assert c["delivered"] == oracle.counts()["delivered"]
    np.testing.assert_array_equal(W.ubench_result(e, w), W.ubench_result(oracle, wo))
