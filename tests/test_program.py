"""Behaviours as programs (GPU_ACTOR_HT_PROGRAM, include/gpu_actor.h) on the CPU:
the assembler's encoding, and the oracle's interpreter (oracle/bsp.c
run_program) against the oracle's compiled tables it restates — the ring and
the deterministic message-ubench ping give the same state, counts and step
counts whether run as a compiled table or as a program. The GPU's interpreter
is checked against this oracle in tests/test_gpu_program.py."""
import numpy as np
import pytest

import pyoracle
from ponyc_amd import program as P
from ponyc_amd import workloads as W
from ponyc_amd.engine import HT_PROGRAM


def run_lossy(e):
    """run(); a SEND past the world's ids is a lost message, which run reports
    as GPU_ACTOR_EMAILBOX after finishing (engine and oracle alike)."""
    try:
        return e.run(), 0
    except Exception as exc:                          # OracleError / GpuActorError
        if getattr(exc, "code", None) != -4:
            raise
        return e.counts()["steps"], -4


def _run(setup, result, lossy=False):
    o = pyoracle.Oracle()
    try:
        w = setup(o)
        steps = run_lossy(o)[0] if lossy else o.run()
        return steps, o.counts(), result(o, w)
    finally:
        o.shutdown()


def test_encoding():
    w = P.word(P.OPS["addi"], 3, 4, 5, -2)
    assert w & 0xFF == 13 and (w >> 8) & 15 == 3 and (w >> 12) & 15 == 4 and (w >> 16) & 15 == 5
    assert (w >> 32) == 0xFFFFFFFE
    p = P.Program()
    p.behaviour(2)
    p.label("top")
    p.jmp("top")
    code = p.assemble()
    assert code[2] == 16 and len(code) == 17
    assert int(code[16]) >> 32 == 0xFFFFFFFF          # pc += -1: the jump itself
    with pytest.raises(ValueError):
        P.word(1, 16)


@pytest.mark.parametrize("size,count,passes", [(3, 1, 10), (64, 4, 100), (1, 2, 5)])
def test_ring_program_equals_compiled(size, count, passes):
    sc, cc, rc = _run(lambda e: W.ring(e, size, count, passes), W.ring_result)
    sp, cp, rp = _run(lambda e: W.ring_prog(e, size, count, passes),
                      lambda e, w: e.state_read(w["type"])[2:4])
    assert sp == sc
    np.testing.assert_array_equal(rp, rc)
    for k in ("delivered", "sent", "pending", "dropped"):
        assert cp[k] == cc[k], k


@pytest.mark.parametrize("n,initial,hops,batch", [(1000, 5, 9, 0), (300, 8, 12, 3)])
def test_det_program_equals_compiled(n, initial, hops, batch):
    sc, cc, rc = _run(lambda e: W.ubench(e, n, initial, det=True, hops=hops, batch=batch),
                      W.ubench_result)
    sp, cp, rp = _run(lambda e: W.det_prog(e, n, initial, hops, batch=batch),
                      lambda e, w: e.state_read(w["type"])[0:2])
    assert sp == sc
    np.testing.assert_array_equal(rp, rc)
    for k in ("delivered", "sent", "pending", "dropped"):
        assert cp[k] == cc[k], k


@pytest.mark.parametrize("count", [1, 2, 6, 10])
def test_spreader_program_equals_compiled(count):
    """The SPAWN op (pony_create + the constructor message inside a
    behaviour): the spreader as a program builds the same tree — every node's
    state, the ids it gets, the counts and the step count — as the compiled
    GPU_ACTOR_HT_SPREADER table."""
    sc, cc, rc = _run(lambda e: W.spreader(e, count), W.spreader_result)
    sp, cp, rp = _run(lambda e: W.spreader_prog(e, count),
                      lambda e, w: e.state_read(w["type"])[0:5])
    assert sp == sc
    np.testing.assert_array_equal(rp, rc)
    for k in ("delivered", "sent", "pending", "dropped"):
        assert cp[k] == cc[k], k


def edge_program() -> np.ndarray:
    """Behaviour 0: r0 += 1, a send past the world's ids (dropped), yield.
    Behaviour 1: a loop that never ends (stops after MAX_STEPS instructions,
    r1 counting its iterations). Behaviour 2: an unknown op ends it before r2
    changes. Behaviour 3: a jump out of the program ends it."""
    p = P.Program()
    p.behaviour(0)
    p.addi(0, 0, 1)
    p.ldi(11, -1)
    p.send(11, 0, 8)
    p.yield_()
    p.halt()
    p.behaviour(1)
    p.label("loop")
    p.addi(1, 1, 1)
    p.jmp("loop")
    p.behaviour(2)
    p.raw(0xFE)
    p.addi(2, 2, 1)
    p.halt()
    p.behaviour(3)
    p.addi(3, 3, 7)
    p.raw(P.word(P.OPS["jmp"], imm=1000))
    p.addi(3, 3, 1)
    return p.assemble()


def edges(e, n=64, k=4):
    e.type_register(0, 8, HT_PROGRAM)
    e.type_config(0, 2, 0)
    e.type_program(0, edge_program())
    first = e.create(0, n)
    i = np.arange(n, dtype=np.uint64) + np.uint64(first)
    m = np.concatenate([W._msgs(i, b, 5) for b in range(4) for _ in range(k)])
    W._sendv(e, m)
    return {"type": 0, "first": first, "n": n}


def test_program_edges_in_the_oracle():
    s, c, r = _run(edges, lambda e, w: e.state_read(w["type"]), lossy=True)
    n, k = 64, 4
    assert (r[0] == k).all()
    assert (r[1] == k * (P.MAX_STEPS // 2)).all()      # addi + jmp per iteration
    assert (r[2] == 0).all() and (r[3] == 7 * k).all()
    assert c["dropped"] == n * k and c["delivered"] == 4 * n * k
    assert s >= k                                        # behaviour 0 yields: one per step
