"""GPU parity of behaviours as programs (GPU_ACTOR_HT_PROGRAM): the device
interpreter (engine_dev.h handle<GPU_ACTOR_HT_PROGRAM>) against the oracle's
(oracle/bsp.c run_program), which tests/test_program.py pins to the oracle's
compiled ring and deterministic ping — state words, counts and step counts, at
both zone geometries, with carried mail (batch 3), and the edge cases: a send
past the world's ids (lost, reported as GPU_ACTOR_EMAILBOX), yield, the
instruction budget, an unknown op and a jump out of the program; and the
spreader, whose children come from the SPAWN op. Every case runs both ways:
the step compiled from the programs at run time (csrc/jit_host.h, the
default: PONYC_AMD_JIT=1) and the interpreter (PONYC_AMD_JIT=0)."""
import numpy as np
import pytest

from ponyc_amd import workloads as W
from test_program import edges, run_lossy

pytestmark = pytest.mark.gpu


def _same(engine_factory, oracle, setup, lossy=False, jit=None):
    e = engine_factory()
    we = setup(e)
    se, rce = run_lossy(e) if lossy else (e.run(), 0)
    ge, ce = e.state_read(we["type"]), e.counts()
    wo = setup(oracle)
    so, rco = run_lossy(oracle) if lossy else (oracle.run(), 0)
    go, co = oracle.state_read(wo["type"]), oracle.counts()
    np.testing.assert_array_equal(ge, go)
    for k in ("delivered", "sent", "pending", "dropped"):
        assert ce[k] == co[k], (k, ce[k], co[k])
    assert se == so and rce == rco
    if jit is not None:
        d = e.debug_info()
        # the zone steps ran the compiled module (a run that stayed on the
        # small-step path never needs it)
        assert (d["jit_builds"] >= 1) == (jit == "1" and d["sparse_steps"] < se), d
    return ge, ce


@pytest.mark.parametrize("jit", ["1", "0"])
@pytest.mark.parametrize("bits", ["11", "12"])
@pytest.mark.parametrize("size,count,passes", [(3, 1, 10), (64, 4, 100), (1000, 10, 50)])
def test_ring_program(engine_factory, oracle, monkeypatch, bits, size, count, passes, jit):
    monkeypatch.setenv("PONYC_AMD_ZONE_BITS", bits)
    monkeypatch.setenv("PONYC_AMD_JIT", jit)
    ge, _ = _same(engine_factory, oracle, lambda e: W.ring_prog(e, size, count, passes), jit=jit)
    assert ge[2].sum() == count * (passes + 1)


@pytest.mark.parametrize("jit", ["1", "0"])
@pytest.mark.parametrize("bits", ["11", "12"])
@pytest.mark.parametrize("n,initial,hops,batch", [(9000, 5, 9, 0), (300, 8, 12, 3)])
def test_det_program(engine_factory, oracle, monkeypatch, bits, n, initial, hops, batch, jit):
    monkeypatch.setenv("PONYC_AMD_ZONE_BITS", bits)
    monkeypatch.setenv("PONYC_AMD_JIT", jit)
    _same(engine_factory, oracle, lambda e: W.det_prog(e, n, initial, hops, batch=batch), jit=jit)


@pytest.mark.parametrize("jit", ["1", "0"])
def test_program_edges(engine_factory, oracle, monkeypatch, jit):
    monkeypatch.setenv("PONYC_AMD_JIT", jit)
    _, c = _same(engine_factory, oracle, edges, lossy=True, jit=jit)
    assert c["dropped"] == 64 * 4


@pytest.mark.parametrize("jit", ["1", "0"])
@pytest.mark.parametrize("bits", ["11", "12"])
@pytest.mark.parametrize("count", [2, 8, 12])
def test_spreader_program(engine_factory, oracle, monkeypatch, bits, count, jit):
    """The SPAWN op: the spreader as a program builds the reference's tree —
    every node's state and id — as the oracle does (tests/test_program.py
    pins the oracle's program to its compiled spreader)."""
    monkeypatch.setenv("PONYC_AMD_ZONE_BITS", bits)
    monkeypatch.setenv("PONYC_AMD_JIT", jit)
    ge, _ = _same(engine_factory, oracle, lambda e: W.spreader_prog(e, count), jit=jit)
    assert ge[4][0] == (1 << count) - 1             # the root prints the node count
