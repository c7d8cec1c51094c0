"""Backpressure, yield and hot receivers on the GPU, bit-exact against the
oracle (oracle/bsp.c restates the rules: DESIGN.md §2).

- mute (actor.c:340-381, 898-921; scheduler.c:1496-1635): a send to an
  overloaded or muted actor mutes a sender that is not itself overloaded; the
  sender stops after that behaviour and waits while the receiver stays
  overloaded. examples/overload is the shape: many senders, one receiver.
- yield (ponyint_actor_yield, actor.c:675-679): the run ends after the
  behaviour; the rest of the mail waits, in order.
- hot receivers: an arrival group above kBigGroup is sorted by the whole
  workgroup (zone_dev.h coop_msd_sort), both with the LDS index (<= 16K
  records in the zone) and with records materialised in S.
Every case also checks that nothing was dropped."""
import numpy as np
import pytest

from ponyc_amd import workloads as W

pytestmark = pytest.mark.gpu


def _both(engine_factory, oracle, setup, result, **kw):
    e = engine_factory(**kw)
    we = setup(e)
    se = e.run()
    ce = e.counts()
    re = result(e, we)
    wo = setup(oracle)
    so = oracle.run()
    co = oracle.counts()
    ro = result(oracle, wo)
    np.testing.assert_array_equal(re, ro)
    assert se == so, (se, so)
    assert ce["delivered"] == co["delivered"] and ce["sent"] == co["sent"]
    assert ce["pending"] == co["pending"] == 0
    assert ce["delivered_by_type"] == co["delivered_by_type"]
    assert ce["dropped"] == 0
    return se, ce, re


@pytest.mark.parametrize("sources,sinks,bursts,m,batch", [
    (64, 7, 10, 4, 7),         # sinks overloaded every step: senders mute and wait
    (500, 2, 3, 2, 10),
    (3000, 4, 2, 1, 100),
])
def test_mute_overloaded_sinks(engine_factory, oracle, sources, sinks, bursts, m, batch):
    _both(engine_factory, oracle,
          lambda e: W.fifo(e, sources, sinks, bursts, m, batch=batch, mailbox_cap=16),
          W.fifo_result, mailbox_cap=16)


def test_fanin_100k_to_4_fifo_sinks(engine_factory, oracle):
    """SURVEY C3's shape with non-commutative receivers: 100,000 senders into
    4 FIFO sinks (mailbox_cap 16, batch 100): bursts far past capacity, hot
    groups of ~25,000 sorted by the workgroup, senders muted while the sinks
    are overloaded; bit-exact, zero drops."""
    se, ce, _ = _both(engine_factory, oracle,
                      lambda e: W.fifo(e, 100_000, 4, 2, 1, mailbox_cap=16),
                      W.fifo_result, mailbox_cap=16)
    assert ce["delivered"] == 100_000 * 2 + 100_000 * 2


@pytest.mark.parametrize("every,batch", [(1, 0), (3, 0), (5, 4)])
def test_yield(engine_factory, oracle, every, batch):
    _both(engine_factory, oracle,
          lambda e: W.fifo(e, 40, 3, 4, 5, batch=batch, mailbox_cap=64, sink_yield=every),
          W.fifo_result)


@pytest.mark.parametrize("sources,m", [(5000, 3), (20_000, 2)])
def test_hot_receiver_group_sort(engine_factory, oracle, sources, m):
    """Two sinks take thousands of arrivals each in one step with a batch that
    runs them all: order is the workgroup sort's alone (LDS-index path at
    15,000 records, S path at 40,000)."""
    _both(engine_factory, oracle,
          lambda e: W.fifo(e, sources, 2, 1, m, batch=1 << 20, mailbox_cap=16),
          W.fifo_result, mailbox_cap=16)


@pytest.mark.parametrize("sources,sinks,bursts,m,batch,prio", [
    (64, 7, 10, 4, 7, 1),       # a priority sink drains its whole mailbox every step
    (64, 7, 10, 4, 7, -3),      # a negative priority keeps one batch per step
    (700, 4, 3, 2, 10, 2),      # groups of 350: exactly-full last batches stay overloaded
    (3000, 4, 2, 1, 100, 5),    # 750 arrivals per sink, sorted by the workgroup, run whole
])
def test_priority(engine_factory, oracle, sources, sinks, bursts, m, batch, prio):
    """The fork's _priority() hint (actor.c:414-416; scheduler.c:1053-1068),
    restated per superstep (include/gpu_actor.h gpu_actor_type_priority):
    mute, overload and carry follow from the sinks draining batch after
    batch."""
    _both(engine_factory, oracle,
          lambda e: W.fifo(e, sources, sinks, bursts, m, batch=batch, mailbox_cap=16,
                           sink_priority=prio),
          W.fifo_result, mailbox_cap=16)


@pytest.mark.parametrize("defer", ["0", "1"])
@pytest.mark.parametrize("sources,sinks,bursts,m,batch", [
    (100_000, 4, 2, 1, 100),    # four backlogs of ~25,000, drained 100 a step
    (60_000, 40, 1, 1, 50),     # forty backlogs of 1,500 over one zone
    (574_000, 4100, 1, 1, 5),   # 4,100 backlogs in one step: past the k_carry_big list
    (410_000, 4100, 1, 1, 1000),  # two zones grown 9x in one burst, no carry
    (2048 * 140, 2048, 1, 1, 5),  # one zone grown 14x: the spill lists re-sized after it
])
def test_backlog_copies(engine_factory, oracle, monkeypatch, defer, sources, sinks, bursts, m, batch):
    """Backlogs (remainders above kBigGroup) copied to the next step's carry
    by the zone's own workgroup (PONYC_AMD_DEFER_BIG=0) or listed for
    k_carry_big and copied by every CU (1; past its 4,096-entry list the zone
    copies the rest itself); carried backlogs are then counted from samples
    (zone_dev.h kCarryRun). Bit-exact either way."""
    monkeypatch.setenv("PONYC_AMD_DEFER_BIG", defer)
    _both(engine_factory, oracle,
          lambda e: W.fifo(e, sources, sinks, bursts, m, batch=batch, mailbox_cap=16),
          W.fifo_result, mailbox_cap=16)


@pytest.mark.parametrize("hot", ["0", "1"])
@pytest.mark.parametrize("m", [5, 20, 40])
def test_hot_group_sort_paths(engine_factory, oracle, monkeypatch, m, hot):
    """A hot sink's arrival group sorted by the workgroup (zone_dev.h
    coop_msd_sort): 3000 sources burst m PUSHes each at one sink. The MSD
    pass bins the keys by their top 11 bits — the sender id's high bits — so
    each bin holds 2m items: m=5 sorts its bins in registers (15,000 arrivals:
    the LDS-index path), m=20 in memory (over 16 items; the scratch path, read
    through the sorted items), m=40 takes the LSD sort (bins over 64; the zone
    also grows 4x in the burst). With PONYC_AMD_HOT=1 the zones of 60,000 and
    120,000 arrivals are prepared by k_hot (hot_dev.h: every CU counts,
    places and bin-sorts them; bins of one sender's 20 or 40 records sorted
    in memory) and k_step reads them in place."""
    monkeypatch.setenv("PONYC_AMD_HOT", hot)
    _both(engine_factory, oracle, lambda e: W.fifo(e, 3000, 1, 1, m, mailbox_cap=16),
          W.fifo_result)


def _hot_zones_60_to_70(e):
    """Idle ring actors fill zones 0-59 (type 0); 22,528 FIFO sinks fill zones
    60-70 (type 1); 45,056 sources (type 2) burst 8 PUSHes each, so every
    sink zone lands exactly kHotMin = 32,768 records in one step: eleven hot
    zones, on both sides of the 64-zone wave boundary of k_hot's zone scan."""
    from ponyc_amd.engine import HT_RING
    e.type_register(0, 4, HT_RING)
    e.create(0, 60 * 2048)
    return W.fifo(e, 2 * 11 * 2048, 11 * 2048, 1, 8, sink_type=1, src_type=2, mailbox_cap=16)


def test_hot_zones_past_kmaxhot(engine_factory, oracle, monkeypatch):
    """More hot zones than k_hot prepares in a step (the list was
    filled in the order the waves ran, so workgroups could disagree on it):
    the kMaxHot lowest zone indices go to k_hot in every workgroup, the rest
    to k_step's own path; bit-exact against the oracle."""
    monkeypatch.setenv("PONYC_AMD_HOT", "1")
    made = []

    def factory(**kw):
        e = engine_factory(**kw)
        made.append(e)
        return e
    se, ce, _ = _both(factory, oracle, _hot_zones_60_to_70, W.fifo_result, mailbox_cap=16)
    d = made[0].debug_info()
    assert d["hot_on"] == 1 and d["hot_missed"] == 0
    assert d["jit_builds"] == 1          # the mix's own any-mix step (csrc/jit_host.h)


@pytest.mark.parametrize("shape", ["fanin_100k_4", "zones_60_70"])
def test_hot_missed_phase_falls_back(engine_factory, oracle, monkeypatch, shape):
    """A k_hot workgroup that misses a phase (forced here with
    PONYC_AMD_HOT_TEST=1, as a grid-barrier timeout would) is reported at the
    zone's end; the last workgroup then gives the zone back to k_step, which
    counts, places and sorts it from the landing buffer: bit-exact, and the
    misses are counted (gpu_actor_debug_info hot_missed)."""
    monkeypatch.setenv("PONYC_AMD_HOT", "1")
    monkeypatch.setenv("PONYC_AMD_HOT_TEST", "1")
    made = []

    def factory(**kw):
        e = engine_factory(**kw)
        made.append(e)
        return e
    setup = (_hot_zones_60_to_70 if shape == "zones_60_70"
             else (lambda e: W.fifo(e, 100_000, 4, 2, 1, mailbox_cap=16)))
    _both(factory, oracle, setup, W.fifo_result, mailbox_cap=16)
    d = made[0].debug_info()
    assert d["hot_on"] == 1
    assert d["hot_missed"] > 0
