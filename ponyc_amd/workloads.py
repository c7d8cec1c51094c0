"""The BASELINE workloads as gpu_actor programs: the host side of each example's
`Main` actor (actor graph construction + initial sends), restated over the
engine interface. Each setup works on any object with the Engine interface
(ponyc_amd.engine.Engine, or the test oracle), so parity tests drive both with
the same code.

Reference programs: examples/ring, examples/message-ubench, examples/fan-in,
examples/gups_basic.
"""
from __future__ import annotations

import numpy as np

from .engine import (MSG_DTYPE, HT_RING, HT_PINGER, HT_PINGER_DET, HT_FANIN_SENDER,
                     HT_FANIN_ANALYZER, HT_GUPS_STREAMER, HT_GUPS_UPDATER, HT_STORM,
                     HT_FIFO_SRC, HT_FIFO_SINK, RING_SET, RING_PASS, PINGER_PING,
                     FANIN_SEND_MSGS, GUPS_APPLY, STORM_TOKEN, STORM_STORM, FIFO_BURST,
                     HT_SPREADER, SPREADER_SPREAD, HT_PROGRAM, NONE_ID)
from . import program as P


def _msgs(to, beh, arg) -> np.ndarray:
    to = np.asarray(to, dtype=np.uint64)
    out = np.empty(to.shape[0], dtype=MSG_DTYPE)
    out["to"] = to.astype(np.uint32)
    out["behaviour"] = np.broadcast_to(np.asarray(beh, dtype=np.uint32), to.shape)
    out["arg"] = np.broadcast_to(np.asarray(arg, dtype=np.uint64), to.shape)
    return out


def _sendv(eng, m: np.ndarray) -> None:
    """Each rank runs the same Main and injects its own share: the messages
    addressed to actors it owns (id % n_ranks == rank); the C-ABI rejects the
    others (include/gpu_actor.h, gpu_actor_sendv)."""
    r = getattr(eng, "n_ranks", 1)
    if r > 1:
        m = m[(m["to"].astype(np.uint64) % np.uint64(r)) == np.uint64(eng.rank)]
    eng.sendv(m)


def _send(eng, to: int, beh: int, arg: int) -> None:
    r = getattr(eng, "n_ranks", 1)
    if r == 1 or to % r == eng.rank:
        eng.send(to, beh, arg)


# ---- examples/ring ---------------------------------------------------------------
def ring(eng, size: int, count: int, passes: int, type_id: int = 0) -> dict:
    """setup_ring (ring/main.pony:61-72): `count` rings of `size` actors; actor 1
    of each ring gets set(actor 2) then pass(passes)."""
    eng.type_register(type_id, 4, HT_RING)
    eng.type_param(type_id, 0, size)
    first = eng.create(type_id, size * count)
    j = np.arange(count, dtype=np.uint64)
    heads = first + j * size
    nxt = heads + (1 % size)
    m = np.empty(2 * count, dtype=MSG_DTYPE)
    m[0::2] = _msgs(heads, RING_SET, nxt)
    m[1::2] = _msgs(heads, RING_PASS, passes)
    if passes == 0:
        m = m[0::2]
    _sendv(eng, m)
    return {"type": type_id, "first": first, "n": size * count,
            "total_msgs": count * (passes + 1) + count}


def ring_result(eng, w: dict) -> np.ndarray:
    """[recv, done] per actor (index = ring*size + id-1)."""
    return eng.state_read(w["type"])[2:4]


def ring_prog(eng, size: int, count: int, passes: int, type_id: int = 0) -> dict:
    """`ring` with the ring's behaviours as a program (GPU_ACTOR_HT_PROGRAM,
    ponyc_amd.program.ring_program): the compiled table's constructor state
    (engine.hip k_construct) written by the host, then the same sends."""
    eng.type_register(type_id, 8, HT_PROGRAM)
    eng.type_program(type_id, P.ring_program())
    first = eng.create(type_id, size * count)
    i = np.arange(size * count, dtype=np.uint64)
    ring_i, pos = i // np.uint64(size), i % np.uint64(size)
    st = np.zeros((8, size * count), dtype=np.uint64)
    st[0] = np.where(pos == 0, np.uint64(NONE_ID),
                     np.uint64(first) + ring_i * np.uint64(size) + (pos + np.uint64(1)) % np.uint64(size))
    st[1] = pos + np.uint64(1)
    # each rank writes the actors it owns (id % n_ranks == rank), in id order
    r = getattr(eng, "n_ranks", 1)
    if r > 1:
        st = st[:, ((np.uint64(first) + i) % np.uint64(r)) == np.uint64(eng.rank)]
    eng.state_write(type_id, st)
    heads = first + np.arange(count, dtype=np.uint64) * np.uint64(size)
    m = np.empty(2 * count, dtype=MSG_DTYPE)
    m[0::2] = _msgs(heads, RING_SET, heads + np.uint64(1 % size))
    m[1::2] = _msgs(heads, RING_PASS, passes)
    if passes == 0:
        m = m[0::2]
    _sendv(eng, m)
    return {"type": type_id, "first": first, "n": size * count}


def det_prog(eng, n: int, initial: int = 5, hops: int = 32, seed: int = 5489,
             type_id: int = 0, batch: int = 0, mailbox_cap: int = 0) -> dict:
    """`ubench(det=True)` with the ping as a program (ponyc_amd.program.det_program)."""
    eng.type_register(type_id, 8, HT_PROGRAM)
    if batch or mailbox_cap:
        eng.type_config(type_id, batch, mailbox_cap)
    eng.type_program(type_id, P.det_program(PINGER_PING))
    eng.type_param(type_id, 0, n)
    eng.type_param(type_id, 2, hops)
    eng.type_param(type_id, 3, seed)
    first = eng.create(type_id, n)
    eng.type_param(type_id, 1, first)
    i = np.arange(n, dtype=np.uint64)
    parts = [_msgs(first + i, PINGER_PING, (i * np.uint64(initial) + np.uint64(k)) << np.uint64(32))
             for k in range(initial)]
    _sendv(eng, np.concatenate(parts) if parts else np.empty(0, dtype=MSG_DTYPE))
    return {"type": type_id, "first": first, "n": n}


# ---- examples/message-ubench -------------------------------------------------------
def ubench(eng, n: int, initial: int = 5, budget: int = 100, seed: int = 5489,
           det: bool = False, hops: int = 32, type_id: int = 0, batch: int = 0,
           mailbox_cap: int = 0) -> dict:
    """SyncLeader + n Pingers (message-ubench/main.pony:94-286). Faithful form:
    seeded xoroshiro128+, forward budget per pinger. det: token routing."""
    ht = HT_PINGER_DET if det else HT_PINGER
    eng.type_register(type_id, 2 if det else 3, ht)
    if batch or mailbox_cap:
        eng.type_config(type_id, batch, mailbox_cap)
    eng.type_param(type_id, 0, n)
    eng.type_param(type_id, 2, hops if det else budget)
    eng.type_param(type_id, 3, seed)
    first = eng.create(type_id, n)
    eng.type_param(type_id, 1, first)
    # tell_all_to_go (main.pony:201-218): `initial` rounds over all pingers
    i = np.arange(n, dtype=np.uint64)
    parts = []
    for k in range(initial):
        if det:
            payload = (i * np.uint64(initial) + np.uint64(k)) << np.uint64(32)
        else:
            payload = np.uint64(42)
        parts.append(_msgs(first + i, PINGER_PING, payload))
    _sendv(eng, np.concatenate(parts) if parts else np.empty(0, dtype=MSG_DTYPE))
    return {"type": type_id, "first": first, "n": n, "det": det}


def ubench_result(eng, w: dict) -> np.ndarray:
    """faithful: [x, y, count]; det: [count, acc]."""
    return eng.state_read(w["type"])


# ---- examples/fan-in ------------------------------------------------------------------
def fanin(eng, senders: int, analyzers: int, msgs: int, seedmode: int = 0,
          an_type: int = 0, snd_type: int = 1) -> dict:
    """Coordinator's graph (fan-in/main.pony:114-139): analyzers, then senders
    whose constructor sends send_msgs() to itself."""
    eng.type_register(an_type, 2, HT_FANIN_ANALYZER)
    afirst = eng.create(an_type, analyzers)
    eng.type_register(snd_type, 4, HT_FANIN_SENDER)
    eng.type_param(snd_type, 0, analyzers)
    eng.type_param(snd_type, 1, afirst)
    eng.type_param(snd_type, 2, msgs)
    eng.type_param(snd_type, 3, seedmode)
    sfirst = eng.create(snd_type, senders)
    _sendv(eng, _msgs(sfirst + np.arange(senders, dtype=np.uint64), FANIN_SEND_MSGS, 0))
    return {"an_type": an_type, "snd_type": snd_type, "afirst": afirst, "sfirst": sfirst,
            "total_msgs": 2 * senders * msgs}


def fanin_result(eng, w: dict) -> np.ndarray:
    return eng.state_read(w["an_type"])


# ---- examples/gups_basic ------------------------------------------------------------------
def gups(eng, logtable: int = 20, updaters: int = 8, streamers: int = 4, chunk: int = 1024,
         iterate: int = 10000, up_type: int = 0, str_type: int = 1) -> dict:
    """gups_basic Main (main.pony:40-75): updaters hold table slices, streamers
    stream PolyRand data; one message per update."""
    size = (1 << logtable) // updaters
    eng.type_register(up_type, size, HT_GUPS_UPDATER)
    eng.type_param(up_type, 0, size)
    ufirst = eng.create(up_type, updaters)
    shift = size.bit_length()          # size.bitwidth() - size.clz() (main.pony:102)
    eng.type_register(str_type, 2, HT_GUPS_STREAMER)
    eng.type_param(str_type, 0, chunk)
    eng.type_param(str_type, 1, shift)
    eng.type_param(str_type, 2, updaters - 1)
    eng.type_param(str_type, 3, ufirst)
    eng.type_param(str_type, 5, chunk * iterate)
    sfirst = eng.create(str_type, streamers)
    _sendv(eng, _msgs(sfirst + np.arange(streamers, dtype=np.uint64), GUPS_APPLY, iterate))
    return {"up_type": up_type, "str_type": str_type, "size": size, "updaters": updaters,
            "updates": streamers * chunk * (iterate + 1)}


def gups_result(eng, w: dict) -> np.ndarray:
    """Whole table, updater-major (as harness_gups writes it)."""
    st = eng.state_read(w["up_type"])          # [size][updaters_local]
    return np.ascontiguousarray(st.T).reshape(-1)


# ---- synthetic storm (C5) -------------------------------------------------------------------
def storm(eng, n: int, r: int = 4, hops: int = 16, seed: int = 5489, type_id: int = 0,
          mailbox_cap: int = 0) -> dict:
    eng.type_register(type_id, 2, HT_STORM)
    if mailbox_cap:
        eng.type_config(type_id, 0, mailbox_cap)
    eng.type_param(type_id, 0, n)
    eng.type_param(type_id, 2, hops)
    eng.type_param(type_id, 3, seed)
    first = eng.create(type_id, n)
    eng.type_param(type_id, 1, first)
    i = np.arange(n, dtype=np.uint64)
    parts = [_msgs(first + i, STORM_TOKEN, 0)]
    for k in range(r):
        parts.append(_msgs(first + i, STORM_STORM,
                           (i * np.uint64(r) + np.uint64(k)) << np.uint64(32)))
    _sendv(eng, np.concatenate(parts))
    return {"type": type_id, "first": first, "n": n}


# ---- examples/spreader ---------------------------------------------------------------------
def spreader(eng, count: int = 10, type_id: int = 0) -> dict:
    """Main + Spreader(env) (spreader/main.pony:50-52, 9-19): one root actor;
    every node spawns two children until count reaches 1, so the tree has
    2^count - 1 actors, all but the root spawned by behaviours."""
    eng.type_register(type_id, 5, HT_SPREADER)
    nodes = (1 << count) - 1
    eng.type_reserve(type_id, nodes - 1)
    root = eng.create(type_id, 1)
    _send(eng, root, SPREADER_SPREAD, (0xFFFFFFFF << 32) | count)
    return {"type": type_id, "root": root, "nodes": nodes}


def spreader_prog(eng, count: int = 10, type_id: int = 0) -> dict:
    """`spreader` with the Spreader's behaviours as a program
    (ponyc_amd.program.spreader_program): the children are created by the
    program's SPAWN op."""
    eng.type_register(type_id, 8, HT_PROGRAM)
    eng.type_program(type_id, P.spreader_program(type_id))
    nodes = (1 << count) - 1
    eng.type_reserve(type_id, nodes - 1)
    root = eng.create(type_id, 1)
    _send(eng, root, SPREADER_SPREAD, (0xFFFFFFFF << 32) | count)
    return {"type": type_id, "root": root, "nodes": nodes}


def spreader_result(eng, w: dict) -> np.ndarray:
    """[count, parent, _result, _received, printed] of every actor, by id."""
    return eng.state_read(w["type"])


# ---- per-pair FIFO probe ---------------------------------------------------------------------
def fifo(eng, sources: int = 64, sinks: int = 8, bursts: int = 10, m: int = 4,
         sink_type: int = 0, src_type: int = 1, batch: int = 0, mailbox_cap: int = 0,
         sink_yield: int = 0, sink_priority: int = 0) -> dict:
    """Per-pair FIFO probe (include/gpu_actor.h HT_FIFO_SRC/SINK): `sources`
    actors burst m PUSHes each to sink i % sinks, `bursts` times. The sink's
    fold is order-sensitive; `sink_yield` > 0 makes it yield after every k-th
    message (ponyint_actor_yield); `sink_priority` is the sinks' _priority()
    hint. The shape of examples/overload (many senders, one slow receiver)
    when sources >> sinks."""
    eng.type_register(sink_type, 11, HT_FIFO_SINK)
    if batch or mailbox_cap:
        eng.type_config(sink_type, batch, mailbox_cap)
    eng.type_param(sink_type, 0, sinks)
    eng.type_param(sink_type, 1, sink_yield)
    if sink_priority:
        eng.type_priority(sink_type, sink_priority)
    kfirst = eng.create(sink_type, sinks)
    eng.type_register(src_type, 3, HT_FIFO_SRC)
    eng.type_param(src_type, 0, kfirst)
    eng.type_param(src_type, 1, sinks)
    eng.type_param(src_type, 2, bursts)
    sfirst = eng.create(src_type, sources)
    _sendv(eng, _msgs(sfirst + np.arange(sources, dtype=np.uint64), FIFO_BURST, m))
    return {"sink_type": sink_type, "src_type": src_type}


def fifo_result(eng, w: dict) -> np.ndarray:
    return eng.state_read(w["sink_type"])
