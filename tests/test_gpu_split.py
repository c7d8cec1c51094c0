"""GPU parity of the step run as one launch or as two.

A two-pass table's step (the message-ubench pinger) is two launches by default
(zone_dev.h k_step PM 1: the zones that take the two passes; PM 2: the rest,
on the general path); so is C2-det's and the storm's (PM 1: the plain zones —
no carried mail, no backpressure, no group over kBigGroup; PM 2: the rest).
PONYC_AMD_SPLIT_PLAN=0 runs the one-launch kernel (PM 0). Both must equal the
oracle: steps where every zone takes PM 1, steps where the batch limit, carried
mail or a hot group send zones to PM 2, and a forward budget whose ramp-down
mixes the two in one step — at both zone geometries."""
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


@pytest.mark.parametrize("bits", ["11", "12"])
@pytest.mark.parametrize("split", ["0", "1"])
@pytest.mark.parametrize("name", list(CASES))
def test_split_launch(engine_factory, oracle, monkeypatch, name, split, bits):
    monkeypatch.setenv("PONYC_AMD_SPLIT_PLAN", split)
    monkeypatch.setenv("PONYC_AMD_ZONE_BITS", bits)
    setup, result = CASES[name]
    g, o = _both(engine_factory, oracle, setup, result)
    _assert_same(g, o)
