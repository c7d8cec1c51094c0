"""The priority rule of the CPU restatement (oracle/bsp.c run_step;
include/gpu_actor.h gpu_actor_type_priority), checked on its own terms: the
reference schedules priorities by thread timing, so no fixture pins it
(parity with the reference unpinned; the GPU engine is checked against this
rule in tests/test_gpu_backpressure.py::test_priority)."""
import numpy as np

import pyoracle
from ponyc_amd import workloads as W


def _run(prio, batch=7):
    with pyoracle.Oracle() as o:
        w = W.fifo(o, 64, 7, 10, 4, batch=batch, mailbox_cap=16, sink_priority=prio)
        steps = o.run()
        return steps, o.counts(), W.fifo_result(o, w)


def test_priority_drains_the_whole_mailbox_each_step():
    s0, c0, r0 = _run(0)
    s1, c1, r1 = _run(1)
    assert c0["delivered"] == c1["delivered"] and c0["pending"] == c1["pending"] == 0
    assert s1 < s0                       # the sinks never carry mail over
    # every sink saw every message (state word 0, one column per sink),
    # whatever the interleaving
    np.testing.assert_array_equal(r0[0], r1[0])


def test_non_positive_priority_is_the_default():
    s0, c0, r0 = _run(0)
    sm, cm, rm = _run(-3)
    assert s0 == sm and c0 == cm
    np.testing.assert_array_equal(r0, rm)
