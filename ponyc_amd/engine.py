"""Python host binding of libgpuactor.so (the C-ABI in include/gpu_actor.h).

This is the host-side mirror of the reference's runtime interface for the hot
path (pony.h: pony_init/pony_create/pony_sendv/pony_start):
same call shapes, ids instead of pointers, error codes turned into exceptions.
It loads the in-tree HIP build and fails loudly when it is missing; there is no
CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# PONYC_AMD_LIB selects another in-tree build (e.g. the stamps diagnostic)
LIB_PATH = os.environ.get("PONYC_AMD_LIB", os.path.join(_HERE, "libgpuactor.so"))

MSG_DTYPE = np.dtype([("to", "<u4"), ("behaviour", "<u4"), ("arg", "<u8")])
MAX_TYPES = 16

# handler tables / behaviours (include/gpu_actor.h)
HT_RING, HT_PINGER, HT_PINGER_DET, HT_FANIN_SENDER, HT_FANIN_ANALYZER = 1, 2, 3, 4, 5
HT_GUPS_STREAMER, HT_GUPS_UPDATER, HT_STORM, HT_FIFO_SRC, HT_FIFO_SINK = 6, 7, 8, 9, 10
RING_SET, RING_PASS = 0, 1
PINGER_PING = 0
FANIN_SEND_MSGS, FANIN_MSG = 0, 0
GUPS_APPLY, GUPS_UPDATE = 0, 0
STORM_TOKEN, STORM_STORM = 0, 1
FIFO_BURST, FIFO_PUSH = 0, 0
HT_SPREADER = 11
HT_PROGRAM = 12                 # behaviours as programs (ponyc_amd.program)
SPREADER_SPREAD, SPREADER_RESULT = 0, 1
NONE_ID = 0xFFFFFFFFFFFFFFFF

ERRORS = {
    -1: "EINVAL", -2: "ENOMEM", -3: "ENODEV", -4: "EMAILBOX", -5: "EHIP",
    -6: "ESTATE", -7: "ERANGE", -8: "ECOMM", -9: "EBUSY",
}


class GpuActorError(RuntimeError):
    def __init__(self, fn: str, code: int):
        super().__init__(f"{fn} failed: {ERRORS.get(code, code)} ({code})")
        self.fn = fn
        self.code = code

    def __reduce__(self):              # (crosses process pools)
        return (GpuActorError, (self.fn, self.code))


class Config(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("n_ranks", ctypes.c_uint32),
        ("rank", ctypes.c_uint32),
        ("batch", ctypes.c_uint32),
        ("mailbox_cap", ctypes.c_uint32),
        ("max_exchange", ctypes.c_uint32),
        ("max_actors", ctypes.c_uint64),
        ("comm_id", ctypes.c_void_p),
    ]


class Counts(ctypes.Structure):
    _fields_ = [
        ("steps", ctypes.c_uint64),
        ("delivered", ctypes.c_uint64),
        ("sent", ctypes.c_uint64),
        ("pending", ctypes.c_uint64),
        ("dropped", ctypes.c_uint64),
        ("remote", ctypes.c_uint64),
        ("active", ctypes.c_uint64),
        ("delivered_by_type", ctypes.c_uint64 * MAX_TYPES),
        ("atomics", ctypes.c_uint64),
    ]


# every symbol include/gpu_actor.h declares
EXPORTS = [
    "gpu_actor_init", "gpu_actor_shutdown", "gpu_actor_comm_id",
    "gpu_actor_type_register", "gpu_actor_type_config", "gpu_actor_type_priority",
    "gpu_actor_type_param", "gpu_actor_type_program",
    "gpu_actor_create", "gpu_actor_type_reserve", "gpu_actor_type_live",
    "gpu_actor_alloc_msgs", "gpu_actor_sendv", "gpu_actor_send",
    "gpu_actor_run", "gpu_actor_run_fixed", "gpu_actor_sync",
    "gpu_actor_state_read", "gpu_actor_state_write", "gpu_actor_counts",
    "gpu_actor_owner", "gpu_actor_stream", "gpu_actor_last_drain_ms", "gpu_actor_strerror",
    "gpu_actor_set_transport", "gpu_actor_run_async", "gpu_actor_wait", "gpu_actor_busy",
]

# host-transport callbacks (include/gpu_actor.h: gpu_actor_alltoallv_fn / _allreduce_fn)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_uint64))
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64)
# completion callback of gpu_actor_run_async (include/gpu_actor.h: gpu_actor_done_fn)
DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64)

_lib = None
# set while a run_async completion callback runs on the library's thread
_IN_CALLBACK = threading.local()


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libgpuactor.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} is missing: build it with `python -m ponyc_amd.build` "
            "(the engine has no CPU fallback)")
    lib = ctypes.CDLL(path)
    u32, u64, i32, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p
    sig = {
        "gpu_actor_init": (i32, [ctypes.POINTER(Config)]),
        "gpu_actor_shutdown": (i32, []),
        "gpu_actor_comm_id": (i32, [vp]),
        "gpu_actor_type_register": (i32, [u32, u32, u32]),
        "gpu_actor_type_config": (i32, [u32, u32, u32]),
        "gpu_actor_type_priority": (i32, [u32, ctypes.c_int32]),
        "gpu_actor_type_param": (i32, [u32, u32, u64]),
        "gpu_actor_type_program": (i32, [u32, vp, u32]),
        "gpu_actor_create": (i32, [u32, u64, ctypes.POINTER(u64)]),
        "gpu_actor_type_reserve": (i32, [u32, u64]),
        "gpu_actor_type_live": (i32, [u32, ctypes.POINTER(u64)]),
        "gpu_actor_alloc_msgs": (i32, [u64, ctypes.POINTER(vp)]),
        "gpu_actor_sendv": (i32, [vp, u64]),
        "gpu_actor_send": (i32, [u64, u32, u64]),
        "gpu_actor_run": (i32, [u64, ctypes.POINTER(u64)]),
        "gpu_actor_run_fixed": (i32, [u64]),
        "gpu_actor_sync": (i32, []),
        "gpu_actor_state_read": (i32, [u32, u64, u64, vp]),
        "gpu_actor_state_write": (i32, [u32, u64, u64, vp]),
        "gpu_actor_counts": (i32, [ctypes.POINTER(Counts)]),
        "gpu_actor_owner": (u32, [u64]),
        "gpu_actor_stream": (vp, []),
        "gpu_actor_last_drain_ms": (ctypes.c_double, []),
        "gpu_actor_strerror": (ctypes.c_char_p, [i32]),
        "gpu_actor_set_transport": (i32, [ALLTOALLV_FN, ALLREDUCE_FN, vp]),
        "gpu_actor_run_async": (i32, [u64, DONE_FN, vp]),
        "gpu_actor_wait": (i32, [ctypes.POINTER(u64)]),
        "gpu_actor_busy": (i32, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _wrap_transport(t):
    """C callbacks around a Python transport; returned so the caller keeps them alive."""
    def _view(ptr, nbytes):
        if nbytes == 0 or not ptr:
            return np.zeros(0, np.uint8)
        return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(ptr))

    def a2a(_ctx, send, send_bytes, recv, recv_bytes):
        try:
            n = t.world_size
            sb = [int(send_bytes[i]) for i in range(n)]
            rb = [int(recv_bytes[i]) for i in range(n)]
            t.alltoallv(_view(send, sum(sb)), sb, _view(recv, sum(rb)), rb)
            return 0
        except Exception as e:  # never let an exception cross the C boundary
            print(f"gpu_actor transport alltoallv failed: {e!r}")
            return -1

    def ar(_ctx, buf, n):
        try:
            arr = np.ctypeslib.as_array(buf, shape=(int(n),))
            t.allreduce(arr)
            return 0
        except Exception as e:
            print(f"gpu_actor transport allreduce failed: {e!r}")
            return -1

    return ALLTOALLV_FN(a2a), ALLREDUCE_FN(ar)


def _ck(fn: str, rc: int) -> None:
    if rc < 0:
        raise GpuActorError(fn, rc)


def as_msgs(msgs) -> np.ndarray:
    """Accept a MSG_DTYPE array or an iterable of (to, behaviour, arg)."""
    if isinstance(msgs, np.ndarray) and msgs.dtype == MSG_DTYPE:
        return np.ascontiguousarray(msgs)
    arr = np.array([tuple(int(v) for v in m) for m in msgs], dtype=MSG_DTYPE)
    return arr


class Engine:
    """One gpu_actor engine per process (the C library keeps a global runtime,
    as libponyrt does)."""

    def __init__(self, device: int = 0, n_ranks: int = 1, rank: int = 0, batch: int = 0,
                 mailbox_cap: int = 0, max_actors: int = 0, max_exchange: int = 0,
                 comm_id: bytes | None = None, transport=None):
        """`comm_id` selects the RCCL exchange; `transport` (an object with
        `alltoallv(send, send_bytes, recv, recv_bytes)` and `allreduce(buf)`
        over numpy arrays, e.g. `ponyc_amd.dist.GlooTransport`) selects the
        host-staged exchange instead. One of them is required when n_ranks > 1."""
        self.lib = load_library()
        self._xp = None
        if transport is not None:
            self._xp = _wrap_transport(transport)
            _ck("gpu_actor_set_transport", self.lib.gpu_actor_set_transport(*self._xp, None))
        cfg = Config()
        cfg.device = device
        cfg.n_ranks = n_ranks
        cfg.rank = rank
        cfg.batch = batch
        cfg.mailbox_cap = mailbox_cap
        cfg.max_exchange = max_exchange
        cfg.max_actors = max_actors
        self._comm = None
        if comm_id is not None:
            self._comm = ctypes.create_string_buffer(bytes(comm_id), 128)
            cfg.comm_id = ctypes.cast(self._comm, ctypes.c_void_p)
        _ck("gpu_actor_init", self.lib.gpu_actor_init(ctypes.byref(cfg)))
        self.n_ranks = n_ranks
        self.rank = rank
        self.words: dict[int, int] = {}
        self.first: dict[int, int] = {}
        self.count: dict[int, int] = {}
        self.reserve: dict[int, int] = {}
        self._thunks: list = []
        self.alive = True

    @staticmethod
    def comm_id() -> bytes:
        lib = load_library()
        buf = ctypes.create_string_buffer(128)
        _ck("gpu_actor_comm_id", lib.gpu_actor_comm_id(buf))
        return buf.raw

    # -- types / actors ----------------------------------------------------
    def type_register(self, type_id: int, state_words: int, handler_table: int) -> None:
        _ck("gpu_actor_type_register",
            self.lib.gpu_actor_type_register(type_id, state_words, handler_table))
        self.words[type_id] = state_words

    def type_config(self, type_id: int, batch: int = 0, mailbox_cap: int = 0) -> None:
        _ck("gpu_actor_type_config", self.lib.gpu_actor_type_config(type_id, batch, mailbox_cap))

    def type_priority(self, type_id: int, priority: int) -> None:
        """The fork's _priority() hint (include/gpu_actor.h)."""
        _ck("gpu_actor_type_priority", self.lib.gpu_actor_type_priority(type_id, priority))

    def type_param(self, type_id: int, idx: int, value: int) -> None:
        _ck("gpu_actor_type_param",
            self.lib.gpu_actor_type_param(type_id, idx, int(value) & 0xFFFFFFFFFFFFFFFF))

    def type_program(self, type_id: int, code) -> None:
        """The behaviours of a GPU_ACTOR_HT_PROGRAM type (ponyc_amd.program
        assembles them; include/gpu_actor.h has the instruction set)."""
        c = np.ascontiguousarray(code, dtype=np.uint64)
        _ck("gpu_actor_type_program",
            self.lib.gpu_actor_type_program(type_id, c.ctypes.data, c.size))

    def type_reserve(self, type_id: int, n: int) -> None:
        """Room for n actors that behaviours spawn while running."""
        _ck("gpu_actor_type_reserve", self.lib.gpu_actor_type_reserve(type_id, n))
        self.reserve[type_id] = n

    def type_live(self, type_id: int) -> int:
        v = ctypes.c_uint64(0)
        _ck("gpu_actor_type_live", self.lib.gpu_actor_type_live(type_id, ctypes.byref(v)))
        return v.value

    def create(self, type_id: int, count: int) -> int:
        first = ctypes.c_uint64(0)
        _ck("gpu_actor_create", self.lib.gpu_actor_create(type_id, count, ctypes.byref(first)))
        self.first[type_id] = first.value
        self.count[type_id] = count + self.reserve.get(type_id, 0)   # id range incl. reserve
        return first.value

    # -- sending -------------------------------------------------------------
    def sendv(self, msgs) -> None:
        arr = as_msgs(msgs)
        if arr.size == 0:
            return
        _ck("gpu_actor_sendv",
            self.lib.gpu_actor_sendv(arr.ctypes.data_as(ctypes.c_void_p), arr.size))

    def send(self, to: int, behaviour: int, arg: int) -> None:
        _ck("gpu_actor_send",
            self.lib.gpu_actor_send(to, behaviour, int(arg) & 0xFFFFFFFFFFFFFFFF))

    # -- running ---------------------------------------------------------------
    def run(self, max_steps: int = 0) -> int:
        steps = ctypes.c_uint64(0)
        _ck("gpu_actor_run", self.lib.gpu_actor_run(max_steps, ctypes.byref(steps)))
        return steps.value

    def run_async(self, max_steps: int = 0, done=None) -> None:
        """gpu_actor_run on the library's progress thread; done(rc, steps) is
        called on that thread when the run ends (the Pony binding sends a
        completion message to a notify actor from there)."""
        def _cb(_ctx, rc, steps):
            _IN_CALLBACK.active = True
            try:
                if done is not None:
                    done(rc, steps)
            finally:
                _IN_CALLBACK.active = False
        thunk = DONE_FN(_cb)
        rc = self.lib.gpu_actor_run_async(max_steps, thunk, None)
        _ck("gpu_actor_run_async", rc)
        # the progress thread holds this pointer until its run ends: keep every
        # accepted thunk alive until shutdown() (outside a callback) has joined it
        self._thunks.append(thunk)

    def wait(self) -> int:
        """Join the last asynchronous run; returns its step count."""
        steps = ctypes.c_uint64(0)
        _ck("gpu_actor_wait", self.lib.gpu_actor_wait(ctypes.byref(steps)))
        return steps.value

    def busy(self) -> bool:
        return bool(self.lib.gpu_actor_busy())

    def run_fixed(self, n: int) -> None:
        _ck("gpu_actor_run_fixed", self.lib.gpu_actor_run_fixed(n))

    def sync(self) -> None:
        _ck("gpu_actor_sync", self.lib.gpu_actor_sync())

    def last_drain_ms(self) -> float:
        return float(self.lib.gpu_actor_last_drain_ms())

    # -- state / counters ----------------------------------------------------------
    def local_count(self, type_id: int) -> int:
        """Actors of a type owned by this rank (ids first + k*n_ranks + ...)."""
        first, count, r, n = self.first[type_id], self.count[type_id], self.rank, self.n_ranks

        def below(x):
            return (x - r + n - 1) // n if x > r else 0
        return below(first + count) - below(first)

    def state_read(self, type_id: int, first: int = 0, n: int | None = None) -> np.ndarray:
        """Field-major state: out[w, i] = word w of local actor first+i."""
        if n is None:
            n = self.local_count(type_id) - first
        words = self.words[type_id]
        out = np.zeros((words, n), dtype=np.uint64)
        _ck("gpu_actor_state_read",
            self.lib.gpu_actor_state_read(type_id, first, n, out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def state_write(self, type_id: int, values: np.ndarray, first: int = 0) -> None:
        arr = np.ascontiguousarray(values, dtype=np.uint64)
        n = arr.shape[1]
        _ck("gpu_actor_state_write",
            self.lib.gpu_actor_state_write(type_id, first, n, arr.ctypes.data_as(ctypes.c_void_p)))

    def counts(self) -> dict:
        c = Counts()
        _ck("gpu_actor_counts", self.lib.gpu_actor_counts(ctypes.byref(c)))
        return {
            "steps": c.steps, "delivered": c.delivered, "sent": c.sent,
            "pending": c.pending, "dropped": c.dropped, "remote": c.remote,
            "active": c.active,
            "delivered_by_type": [c.delivered_by_type[i] for i in range(MAX_TYPES)],
            "atomics": c.atomics,
        }

    def debug_info(self) -> dict:
        """Engine internals (diagnostic export, not in include/gpu_actor.h)."""
        keys = ["fixups", "sparse_launches", "sparse_steps", "zone_records", "spill_cap", "zones",
                "trig_n0", "trig_n1", "trig_n2", "zone_bits", "hot_missed", "hot_on", "jit",
                "jit_builds", "gups_updates", "gups_atomics", "peer_write"]
        out = (ctypes.c_uint64 * len(keys))()
        fn = self.lib.gpu_actor_debug_info
        fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        fn.restype = ctypes.c_int
        _ck("gpu_actor_debug_info", fn(out, len(keys)))
        return {k: int(out[i]) for i, k in enumerate(keys)}

    def stream(self) -> int:
        return int(self.lib.gpu_actor_stream() or 0)

    def shutdown(self) -> None:
        if self.alive:
            _ck("gpu_actor_shutdown", self.lib.gpu_actor_shutdown())
            self.alive = False
            if not getattr(_IN_CALLBACK, "active", False):
                self._thunks.clear()      # the progress thread has been joined
            if self._xp is not None:  # drop the callbacks before they are freed
                self.lib.gpu_actor_set_transport(ALLTOALLV_FN(), ALLREDUCE_FN(), None)
                self._xp = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.shutdown()


def jit_compile(progs, z12: bool = False, arch: str = "gfx950", lib_path: str | None = None) -> None:
    """Compile the step for a program set (`progs`: [(type id, words), ...])
    into the library's code-object cache without a device (csrc/jit_host.h;
    diagnostic export gpu_actor_debug_jit_compile), so that an engine running
    these programs loads it at once."""
    lib = ctypes.CDLL(lib_path or LIB_PATH)
    fn = lib.gpu_actor_debug_jit_compile
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                   ctypes.c_char_p]
    fn.restype = ctypes.c_int
    types = np.array([t for t, _ in progs], dtype=np.uint32)
    words = np.concatenate([np.asarray(w, dtype=np.uint64) for _, w in progs])
    lens = np.array([len(w) for _, w in progs], dtype=np.uint32)
    _ck("gpu_actor_debug_jit_compile", fn(types.ctypes.data, words.ctypes.data, lens.ctypes.data,
                                          len(progs), int(z12), arch.encode()))


def jit_compile_mix(mask: int, z12: bool = False, arch: str = "gfx950", lib_path: str | None = None) -> None:
    """The same for the any-mix step of a mix of compiled tables (`mask`: bit
    per table id; gpu_actor_debug_jit_compile_mix)."""
    lib = ctypes.CDLL(lib_path or LIB_PATH)
    fn = lib.gpu_actor_debug_jit_compile_mix
    fn.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_char_p]
    fn.restype = ctypes.c_int
    _ck("gpu_actor_debug_jit_compile_mix", fn(mask, int(z12), arch.encode()))
