"""The small-step path (k_sparse, ponyc_amd/csrc/sparse_dev.h) against the zone
path (k_step) and the oracle. Every gpu_actor_run goes through k_sparse while
at most kSpCap (1024) records are pending; GPA_NO_SPARSE=1 forces k_step for
every step, so each case below runs both ways and must agree bit for bit with
each other and with the CPU restatement (state, counts, step counts)."""
import os

import numpy as np
import pytest

from ponyc_amd import workloads as W

pytestmark = pytest.mark.gpu


def _run(engine_factory, setup, result, sparse, steps=0):
    old = os.environ.get("GPA_NO_SPARSE")
    os.environ["GPA_NO_SPARSE"] = "0" if sparse else "1"
    try:
        e = engine_factory()
        w = setup(e)
        s = e.run(steps)
        c = e.counts()
        r = result(e, w).copy()
        e.shutdown()
    finally:
        if old is None:
            os.environ.pop("GPA_NO_SPARSE", None)
        else:
            os.environ["GPA_NO_SPARSE"] = old
    return s, c, r


CASES = {
    # one token per ring: every step is sparse
    "ring_100x1000": (lambda e: W.ring(e, 1000, 100, 300), W.ring_result),
    "ring_one": (lambda e: W.ring(e, 1000, 1, 2500), W.ring_result),
    # 4096 x 4 tokens: starts dense, goes sparse as budgets run out
    "ubench_budget": (lambda e: W.ubench(e, 4096, 4, 8), W.ubench_result),
    "ubench_det": (lambda e: W.ubench(e, 300, 3, det=True, hops=60), W.ubench_result),
    # a reducible receiver: applies from inside the sparse step
    "fanin": (lambda e: W.fanin(e, 200, 3, 30, 1), W.fanin_result),
    # batch 4 with arrivals above it: the sparse path hands those steps back
    "fifo_batch": (lambda e: W.fifo(e, 40, 5, 6, 3, batch=4, mailbox_cap=1024), W.fifo_result),
    "storm": (lambda e: W.storm(e, 200, 2, 40), lambda e, w: e.state_read(w["type"])),
    "gups": (lambda e: W.gups(e, 12, 4, 2, 16, 40), W.gups_result),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_sparse_equals_zone_path_and_oracle(engine_factory, oracle, case):
    setup, result = CASES[case]
    sp = _run(engine_factory, setup, result, True)
    dn = _run(engine_factory, setup, result, False)
    wo = setup(oracle)
    so = oracle.run()
    co = oracle.counts()
    ro = result(oracle, wo)
    for s, c, r in (sp, dn):
        np.testing.assert_array_equal(r, ro)
        assert s == so
        assert c["delivered"] == co["delivered"] and c["sent"] == co["sent"]
        assert c["pending"] == co["pending"] == 0
        assert c["delivered_by_type"] == co["delivered_by_type"]
        assert c["dropped"] == 0
    assert sp[1]["active"] == dn[1]["active"]


def test_sparse_max_steps_resume(engine_factory, oracle):
    """run(k) stops inside the sparse path after exactly k steps and resumes."""
    def setup(e):
        return W.ring(e, 50, 7, 400)
    e = engine_factory()
    we = setup(e)
    total, chunks = 0, 0
    while True:
        s = e.run(37)
        total += s
        chunks += 1
        if s < 37:
            break
        assert e.counts()["pending"] > 0
    wo = setup(oracle)
    assert total == oracle.run()
    np.testing.assert_array_equal(W.ring_result(e, we), W.ring_result(oracle, wo))
    assert chunks > 5


def test_sparse_host_sends_between_runs(engine_factory, oracle):
    def go(e):
        w = W.ring(e, 30, 2, 20)
        e.run(5)
        e.send(w["first"] + 3, W.RING_PASS, 4)
        e.send(w["first"] + 40, W.RING_PASS, 9)
        e.run()
        return W.ring_result(e, w)
    np.testing.assert_array_equal(go(engine_factory()), go(oracle))


# ---- run_async corner cases (thunk lifetime, re-entry) -----------------------
def test_run_async_twice_is_ebusy_without_crash(engine_factory, oracle):
    from ponyc_amd.engine import GpuActorError
    import threading
    e = engine_factory()
    w = W.ubench(e, 4096, 4, det=True, hops=64)
    fired = threading.Event()
    e.run_async(0, lambda rc, steps: fired.set())
    try:
        e.run_async(0, lambda rc, steps: None)
    except GpuActorError as ex:
        assert ex.code == -9                       # EBUSY while the first is in flight
    assert fired.wait(60)
    steps = e.wait()
    wo = W.ubench(oracle, 4096, 4, det=True, hops=64)
    assert steps in (oracle.run(), 0)
    np.testing.assert_array_equal(W.ubench_result(e, w), W.ubench_result(oracle, wo))


def test_run_async_callback_chains_calls(engine_factory, oracle):
    """The completion callback calls back into the library: a second
    run_async, then wait and shutdown from the progress thread itself."""
    import threading
    e = engine_factory()
    W.ring(e, 100, 3, 30)
    done = threading.Event()
    seen = []

    def second(rc, steps):
        seen.append(("second", rc, steps))
        seen.append(("wait", e.wait()))
        e.shutdown()
        done.set()

    def first(rc, steps):
        seen.append(("first", rc, steps))
        e.send(0, W.RING_PASS, 5)                  # more mail, then chain a run
        e.run_async(0, second)

    e.run_async(0, first)
    assert done.wait(60), seen
    assert seen[0][1] == 0 and seen[1][1] == 0
    assert seen[1][2] == 6                          # pass(5) visits 6 actors
    assert not e.alive
