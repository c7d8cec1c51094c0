"""GPU parity with 4096-actor zones (1024-thread workgroups, step_*_z12.hip).

The engine picks that geometry by itself only for large engines (over ~640
buckets of 2048-actor zones: C5's 8M actors in test_gpu_fullsize.py); the
PONYC_AMD_ZONE_BITS hook (engine.hip: pick_zone_bits) forces it here so that
small, oracle-checked workloads run every path of the second geometry —
landing, carry and backpressure, hot groups, the small-step path, spawning
and two ranks' exchange."""
import numpy as np
import pytest

from ponyc_amd import workloads as W
from test_gpu_parity import _both, _assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def zone_bits_12(monkeypatch):
    monkeypatch.setenv("PONYC_AMD_ZONE_BITS", "12")


CASES = {
    "ring": (lambda e: W.ring(e, 64, 4, 100), W.ring_result),
    "ubench": (lambda e: W.ubench(e, 9000, 4, 20), W.ubench_result),
    "ubench_det": (lambda e: W.ubench(e, 9000, 5, det=True, hops=9), W.ubench_result),
    "ubench_batch": (lambda e: W.ubench(e, 512, 40, 60, batch=3), W.ubench_result),
    "det_large_groups": (lambda e: W.ubench(e, 256, 40, det=True, hops=12), W.ubench_result),
    "fanin": (lambda e: W.fanin(e, 5000, 16, 20, 1), W.fanin_result),
    "gups": (lambda e: W.gups(e, 16, 8, 4, 1024, 10), W.gups_result),
    "storm": (lambda e: W.storm(e, 9000, 4, 12), lambda e, w: e.state_read(w["type"])),
    "fifo": (lambda e: W.fifo(e, 64, 8, 10, 4), W.fifo_result),
    "fifo_hot": (lambda e: W.fifo(e, 4, 2, 1, 600, mailbox_cap=2048), W.fifo_result),
    "fifo_batch": (lambda e: W.fifo(e, 300, 3, 4, 9, batch=4, mailbox_cap=1), W.fifo_result),
    "spreader": (lambda e: W.spreader(e, 10), W.spreader_result),
    # a zone of 4096 FIFO sinks grown 14x in one burst, then drained from
    # backlogs of 135 (the spill lists re-sized only after the fixup placed them)
    "backlog": (lambda e: W.fifo(e, 4096 * 140, 4096, 1, 1, batch=5, mailbox_cap=16),
                W.fifo_result),
}


@pytest.mark.parametrize("name", list(CASES))
def test_parity_zones_4096(engine_factory, oracle, name):
    setup, result = CASES[name]
    g, o = _both(engine_factory, oracle, setup, result)
    _assert_same(g, o)
    assert g[1]["debug"]["zones"] >= 1
