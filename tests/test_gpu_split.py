"""GPU parity of the step run as one launch or as two.

A two-pass table's step (the message-ubench pinger) is split (zone_dev.h k_step
PM 1: the zones that take the two passes; PM 2: the rest, on the general
path), by default as one launch that calls PM 2's code for the zones PM 1
leaves (PM 3; PONYC_AMD_FUSE=0: two launches); C2-det's and the storm's are two
launches (PM 1: the plain zones — no carried mail, no backpressure, no group
over kBigGroup; PM 2: the rest). PONYC_AMD_SPLIT_PLAN=0 runs the unsplit kernel
(PM 0). Every form must equal the oracle: steps where every zone takes PM 1, steps where the batch limit, carried
mail or a hot group send zones to PM 2, and a forward budget whose ramp-down
mixes the two in one step — at both zone geometries."""
import numpy as np
import pytest

from ponyc_amd import workloads as W
from test_gpu_parity import _both, _assert_same

pytestmark = pytest.mark.gpu

CASES = {
    # every zone plans until the budget runs out; the tail mixes both paths
    "ubench": (lambda e: W.ubench(e, 9000, 4, 20), W.ubench_result),
    # batch 3 of up to 40 pings: carried mail, zones on the general path
    "ubench_batch": (lambda e: W.ubench(e, 512, 40, 60, batch=3), W.ubench_result),
    # 3 zones of 2048 (or 2 of 4096), a short budget: some zones idle early
    "ubench_tail": (lambda e: W.ubench(e, 5000, 2, 3), W.ubench_result),
    # C2-det: plain zones, then the large-group path of 40 arrivals per actor
    "det": (lambda e: W.ubench(e, 9000, 5, det=True, hops=9), W.ubench_result),
    "det_large_groups": (lambda e: W.ubench(e, 256, 40, det=True, hops=12), W.ubench_result),
    # 200 arrivals per actor: hot groups (PM 2) next to plain zones
    "det_hot": (lambda e: W.ubench(e, 64, 200, det=True, hops=3), W.ubench_result),
    "storm": (lambda e: W.storm(e, 9000, 4, 12), lambda e, w: e.state_read(w["type"])),
}


FORMS = {"unsplit": ("0", "1"), "two_launches": ("1", "0"), "fused": ("1", "1")}


@pytest.mark.parametrize("bits", ["11", "12"])
@pytest.mark.parametrize("form", list(FORMS))
@pytest.mark.parametrize("name", list(CASES))
def test_split_launch(engine_factory, oracle, monkeypatch, name, form, bits):
    if form == "fused" and not name.startswith("ubench"):
        pytest.skip("PM 3 is built for the two-pass table only (step_tu.h split_kernel)")
    split, fuse = FORMS[form]
    monkeypatch.setenv("PONYC_AMD_SPLIT_PLAN", split)
    monkeypatch.setenv("PONYC_AMD_FUSE", fuse)
    monkeypatch.setenv("PONYC_AMD_ZONE_BITS", bits)
    setup, result = CASES[name]
    g, o = _both(engine_factory, oracle, setup, result)
    _assert_same(g, o)


@pytest.mark.parametrize("form", list(FORMS))
def test_trigger_slots_clear_after_triggers_stop(engine_factory, oracle, monkeypatch, form):
    """trig_n (zone_dev.h: read step s's slot, add to s+1's, clear s+2's) goes
    back to 0 once no actor triggers muting — also when zone 0 of the clearing
    step runs in the split's first launch (PM 1 never cleared it,
    so a stale count gated every third step onto the general path). 100 extra
    pings make actor 0 run a full batch in step 0 (overloaded: a trigger, the
    oracle's trig_count); no actor triggers after that, while the budgeted
    pings drain over five more steps in which every zone plans."""
    split, fuse = FORMS[form]
    monkeypatch.setenv("PONYC_AMD_SPLIT_PLAN", split)
    monkeypatch.setenv("PONYC_AMD_FUSE", fuse)

    def setup(e):
        w = W.ubench(e, 4096, 3, 6)
        W._sendv(e, W._msgs(np.full(100, w["first"], dtype=np.uint64), W.PINGER_PING, 42))
        return w

    wo = setup(oracle)
    trace = []
    while oracle.run(1):
        trace.append(oracle.trig_count())
    assert trace[0] > 0 and not any(trace[1:]) and len(trace) >= 5, trace
    e = engine_factory()
    we = setup(e)
    assert e.run() == len(trace)
    d = e.debug_info()
    assert (d["trig_n0"], d["trig_n1"], d["trig_n2"]) == (0, 0, 0), d
    np.testing.assert_array_equal(W.ubench_result(e, we), W.ubench_result(oracle, wo))
    ce, co = e.counts(), oracle.counts()
    assert (ce["delivered"], ce["sent"], ce["pending"]) == (co["delivered"], co["sent"], co["pending"])
