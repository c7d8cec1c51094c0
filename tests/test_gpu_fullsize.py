"""GPU checks at BASELINE.json's full sizes.

Where the CPU restatement finishes in seconds (message-ubench-det at 1M
pingers, fan-in with 100K senders, gups on a 2^20 table) the engine is compared
with it bit for bit. Where it does not (steady-state message-ubench at 1M
pingers, the storm at 8M actors — one GPU's share of C5) the checks are the
size-independent properties the workload has: message conservation, the sum of
per-actor counts, and an XOR checksum of every payload delivered."""
import numpy as np
import pytest

from ponyc_amd import workloads as W

pytestmark = pytest.mark.gpu

MILLION = 1 << 20


def _same_as_oracle(engine_factory, oracle, setup, result):
    e = engine_factory()
    we = setup(e)
    se = e.run()
    ce = e.counts()
    re = result(e, we)
    wo = setup(oracle)
    so = oracle.run()
    co = oracle.counts()
    ro = result(oracle, wo)
    assert ce["dropped"] == 0
    assert se == so
    for k in ("delivered", "sent", "pending", "delivered_by_type"):
        assert ce[k] == co[k], k
    np.testing.assert_array_equal(re, ro)
    return ce


def test_c2_ubench_det_1m(engine_factory, oracle):
    """C2, deterministic form: 1,048,576 pingers x 5 tokens x 4 hops."""
    c = _same_as_oracle(engine_factory, oracle,
                        lambda e: W.ubench(e, MILLION, 5, det=True, hops=3), W.ubench_result)
    assert c["delivered"] == MILLION * 5 * 4


def test_c2_ubench_steady_1m(engine_factory):
    """C2 as benched: 1,048,576 pingers x 5 pings, no forward budget. Every
    step delivers (and forwards) exactly the 5N pings in flight."""
    n, initial, steps = MILLION, 5, 12
    e = engine_factory()
    w = W.ubench(e, n, initial, budget=1 << 62)
    e.run_fixed(steps)
    c = e.counts()
    assert c["dropped"] == 0
    assert c["delivered"] == steps * n * initial
    assert c["sent"] == c["delivered"]
    assert c["pending"] == n * initial
    st = W.ubench_result(e, w)            # [x, y, count]
    assert int(st[2].sum()) == c["delivered"]
    # the xoroshiro128+ streams advanced once per ping handled
    assert int(st[2].max()) < 20 * steps


def test_c2_ubench_steady_1m_vs_oracle(engine_factory, oracle):
    """C2 exactly as bench.py runs it — 1,048,576 pingers x 5 pings, no
    forward budget, a fixed number of supersteps — against the CPU
    restatement: every pinger's xoroshiro128+ state [x, y] (KAT-pinned,
    packages/random/_test.pony:473-493) and count bit for bit, and the
    delivered / sent / pending counts."""
    n, initial, steps = MILLION, 5, 8
    e = engine_factory()
    we = W.ubench(e, n, initial, budget=1 << 62)
    e.run_fixed(steps)
    ce = e.counts()
    re = W.ubench_result(e, we)
    wo = W.ubench(oracle, n, initial, budget=1 << 62)
    oracle.run_fixed(steps)
    co = oracle.counts()
    ro = W.ubench_result(oracle, wo)
    assert ce["dropped"] == 0
    for k in ("delivered", "sent", "pending", "delivered_by_type"):
        assert ce[k] == co[k], k
    assert ce["delivered"] == steps * n * initial
    np.testing.assert_array_equal(re, ro)


def test_c3_fanin_100k(engine_factory, oracle):
    """C3: 100,000 senders -> 4 analyzers x 100 messages (atomic-enqueue
    contention worst case; analyzer counts and XOR folds bit-exact)."""
    c = _same_as_oracle(engine_factory, oracle,
                        lambda e: W.fanin(e, 100_000, 4, 100, 0), W.fanin_result)
    assert c["delivered_by_type"][0] == 100_000 * 100


def test_c4_gups_2p20(engine_factory, oracle):
    """C4 on one GPU: 2^20-entry table over 8 updaters, 4 streamers x 1024
    updates x 1001 iterations."""
    _same_as_oracle(engine_factory, oracle, lambda e: W.gups(e, 20, 8, 4, 1024, 1000),
                    W.gups_result)


def _xor_upto(n: int) -> int:
    """0 ^ 1 ^ ... ^ (n - 1)"""
    m = n - 1
    return [m, 1, m + 1, 0][m % 4] if n > 0 else 0


def test_c4_gups_2p30_2p32(engine_factory):
    """C4 at its stated size: a 2^30-entry u64 table (8 GiB) as
    8 updater shards, 2^32 PolyRand updates t[d & (size-1)] ^= d
    (gups_basic/main.pony:93-216), here 2^18 streamers x 4096 x (3 + 1). The
    whole table's XOR must equal the initial table's XOR (table[k] = k +
    index*size, main.pony:145-155) ^ the XOR of every datum streamed, which
    the oracle's PolyRand restatement computes on the CPU
    (oracle/rng.c or_gups_update_xor, pinned to the literal stream walk and
    to a BSP run in tests/test_oracle_golden.py)."""
    import pyoracle
    logtable, updaters, streamers, chunk, iterate = 30, 8, 1 << 18, 4096, 3
    e = engine_factory()
    w = W.gups(e, logtable, updaters, streamers, chunk, iterate)
    assert w["updates"] == 1 << 32
    steps = e.run()
    c = e.counts()
    assert c["dropped"] == 0 and c["pending"] == 0
    assert steps == iterate + 1
    assert c["delivered_by_type"][w["up_type"]] == 1 << 32
    assert c["delivered_by_type"][w["str_type"]] == streamers * (iterate + 1)
    table = e.state_read(w["up_type"])        # the whole 8 GiB table, one copy
    table_xor = int(np.bitwise_xor.reduce(table.reshape(-1)))
    del table
    want = _xor_upto(1 << logtable) ^ pyoracle.load().or_gups_update_xor(streamers, chunk, iterate)
    assert table_xor == want


@pytest.mark.parametrize("hops", [4, 1000])
def test_c5_storm_8m(engine_factory, hops):
    """C5, one GPU's share: 8M actors, a token ring plus 4 random-target pings
    per actor, `hops` hops each (1000: the stated 1000 steps, 41.9 G
    messages). Conservation and an XOR checksum of every payload."""
    n, r = 8 * MILLION, 4
    e = engine_factory()
    w = W.storm(e, n, r, hops)
    steps = e.run()
    c = e.counts()
    assert c["dropped"] == 0 and c["pending"] == 0
    assert steps == hops + 1
    total = n * (r + 1) * (hops + 1)
    assert c["delivered"] == total
    st = e.state_read(w["type"])          # [count, acc]
    assert int(st[0].sum()) == total
    # tokens: every actor sees hop values 0..hops once
    tok = 0
    for h in range(hops + 1):
        tok ^= h
    tok_all = tok if n % 2 else 0
    # pings: origin o in [0, n*r) carries (o << 32) | h for h = 0..hops
    o = np.arange(n * r, dtype=np.uint64)
    ox = int(np.bitwise_xor.reduce(o << np.uint64(32)))
    ping_all = 0
    for h in range(hops + 1):
        ping_all ^= ox ^ (h if (n * r) % 2 else 0)
    assert int(np.bitwise_xor.reduce(st[1])) == tok_all ^ ping_all


def test_c1_ring_full(engine_factory):
    """C1 at its full size (examples/ring --size 1000 --count 100 --pass 10000):
    the reference's own totals — 1,000,100 `pass` messages, 11 received by the
    first actor of each ring and 10 by every other one, and pass(0) reached
    exactly one actor per ring (the reference harness reproduces these at
    1/2/4/8 scheduler threads)."""
    e = engine_factory()
    w = W.ring(e, 1000, 100, 10000)
    steps = e.run()
    c = e.counts()
    recv, done = W.ring_result(e, w)
    assert c["dropped"] == 0 and c["pending"] == 0
    assert c["delivered"] == 1_000_100 + 100           # + one set per ring
    assert steps == 10_001
    per_ring = recv.reshape(100, 1000)
    assert (per_ring[:, 0] == 11).all() and (per_ring[:, 1:] == 10).all()
    assert int(done.sum()) == 100 and (done.reshape(100, 1000).sum(axis=1) == 1).all()
