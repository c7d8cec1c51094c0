"""TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/_ref/liboracle.so (the
CPU BSP restatement, oracle/bsp.c) and runners for the reference-runtime
harnesses (oracle/_ref/harness_*). Import only from tests/, __graft_entry__.smoke
and bench.py's cpu_baseline leg; the product never imports this module.

`Oracle` exposes the same method names as ponyc_amd.engine.Engine so the
workload setups in ponyc_amd.workloads drive both.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "_ref")
LIB = os.path.join(REF_DIR, "liboracle.so")
MSG_DTYPE = np.dtype([("to", "<u4"), ("behaviour", "<u4"), ("arg", "<u8")])
U64 = 0xFFFFFFFFFFFFFFFF

_lib = None


def build(reference: bool = True) -> None:
    """Compile the restatement (always) and the reference runtime + harnesses
    (when /root/reference is present)."""
    targets = ["oracle"]
    if reference and os.path.isdir("/root/reference/src/libponyrt"):
        targets.append("ref")
    subprocess.run(["make", "-s", "-j8", *targets], cwd=HERE, check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build(reference=False)
    lib = ctypes.CDLL(LIB)
    u32, u64, i32, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p
    sig = {
        "or_init": (i32, [u32]), "or_shutdown": (None, []),
        "or_type_register": (i32, [u32, u32, u32]),
        "or_type_config": (i32, [u32, u32, u32]),
        "or_type_priority": (i32, [u32, ctypes.c_int32]),
        "or_type_param": (i32, [u32, u32, u64]),
        "or_type_program": (i32, [u32, vp, u32]),
        "or_create": (i32, [u32, u64, ctypes.POINTER(u64)]),
        "or_type_reserve": (i32, [u32, u64]),
        "or_type_live": (i32, [u32, ctypes.POINTER(u64)]),
        "or_send": (i32, [u64, u32, u64]), "or_sendv": (i32, [vp, u64]),
        "or_run": (i32, [u64, ctypes.POINTER(u64)]),
        "or_state_read": (i32, [u32, u64, u64, vp]),
        "or_state_write": (i32, [u32, u64, u64, vp]),
        "or_counts": (i32, [vp]), "or_type_delivered": (i32, [u32, vp]),
        "or_mulhi": (u64, [u64, u64]),
        "or_splitmix_mix": (u64, [u64]),
        "or_xoro_next": (u64, [vp]), "or_xoro_create": (None, [vp, u64, u64]),
        "or_rand_int": (u64, [vp, u64]), "or_rand_int_unbiased": (u64, [vp, u64]),
        "or_splitmix_next": (u64, [vp]),
        "or_polyrand_create": (None, [vp, u64]), "or_polyrand_next": (u64, [vp]),
        "or_gups_update_xor": (u64, [u64, u64, u64]),
        "or_gups_update_xor_literal": (u64, [u64, u64, u64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class OracleError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__(f"{fn} failed ({code})")
        self.code = code


def _ck(fn, rc):
    if rc < 0:
        raise OracleError(fn, rc)


class Oracle:
    """Single-threaded BSP restatement with the Engine interface."""

    def __init__(self, **_ignored):
        self.lib = load()
        _ck("or_init", self.lib.or_init(16))
        self.n_ranks, self.rank = 1, 0
        self.words, self.first, self.count = {}, {}, {}
        self.reserve = {}
        self.alive = True

    def type_register(self, type_id, state_words, ht):
        _ck("or_type_register", self.lib.or_type_register(type_id, state_words, ht))
        self.words[type_id] = state_words

    def type_config(self, type_id, batch=0, mailbox_cap=0):
        _ck("or_type_config", self.lib.or_type_config(type_id, batch, mailbox_cap))

    def type_priority(self, type_id, priority):
        _ck("or_type_priority", self.lib.or_type_priority(type_id, priority))

    def type_param(self, type_id, idx, value):
        _ck("or_type_param", self.lib.or_type_param(type_id, idx, int(value) & U64))

    def type_program(self, type_id, code):
        c = np.ascontiguousarray(code, dtype=np.uint64)
        _ck("or_type_program", self.lib.or_type_program(type_id, c.ctypes.data, c.size))

    def type_reserve(self, type_id, n):
        _ck("or_type_reserve", self.lib.or_type_reserve(type_id, n))
        self.reserve[type_id] = n

    def type_live(self, type_id):
        v = ctypes.c_uint64(0)
        _ck("or_type_live", self.lib.or_type_live(type_id, ctypes.byref(v)))
        return v.value

    def create(self, type_id, count):
        first = ctypes.c_uint64(0)
        _ck("or_create", self.lib.or_create(type_id, count, ctypes.byref(first)))
        self.first[type_id] = first.value
        self.count[type_id] = count + self.reserve.get(type_id, 0)
        return first.value

    def sendv(self, msgs):
        arr = msgs if isinstance(msgs, np.ndarray) else np.array(
            [tuple(int(v) for v in m) for m in msgs], dtype=MSG_DTYPE)
        arr = np.ascontiguousarray(arr)
        if arr.size:
            _ck("or_sendv", self.lib.or_sendv(arr.ctypes.data_as(ctypes.c_void_p), arr.size))

    def send(self, to, behaviour, arg):
        _ck("or_send", self.lib.or_send(to, behaviour, int(arg) & U64))

    def run(self, max_steps=0):
        steps = ctypes.c_uint64(0)
        rc = self.lib.or_run(max_steps, ctypes.byref(steps))
        _ck("or_run", rc)
        return steps.value

    def run_fixed(self, n):
        self.run(n)

    def local_count(self, type_id):
        return self.count[type_id]

    def state_read(self, type_id, first=0, n=None):
        if n is None:
            n = self.count[type_id] - first
        out = np.zeros((self.words[type_id], n), dtype=np.uint64)
        _ck("or_state_read", self.lib.or_state_read(type_id, first, n,
                                                    out.ctypes.data_as(ctypes.c_void_p)))
        return out

    def state_write(self, type_id, values, first=0):
        arr = np.ascontiguousarray(values, dtype=np.uint64)
        _ck("or_state_write", self.lib.or_state_write(type_id, first, arr.shape[1],
                                                      arr.ctypes.data_as(ctypes.c_void_p)))

    def trig_count(self) -> int:
        """Actors the last step left overloaded or muted."""
        fn = self.lib.or_trig_count
        fn.restype = ctypes.c_uint64
        return int(fn())

    def counts(self):
        c = (ctypes.c_uint64 * 5)()
        self.lib.or_counts(c)
        by_type = []
        for t in range(16):
            v = ctypes.c_uint64(0)
            self.lib.or_type_delivered(t, ctypes.byref(v))
            by_type.append(v.value)
        return {"steps": c[0], "delivered": c[1], "sent": c[2], "pending": c[3],
                "dropped": c[4], "remote": 0, "delivered_by_type": by_type}

    def shutdown(self):
        if self.alive:
            self.lib.or_shutdown()
            self.alive = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.shutdown()


# ---- reference-runtime harnesses ------------------------------------------------

def harness_path(name: str) -> str:
    return os.path.join(REF_DIR, f"harness_{name}")


def run_harness(name: str, args: dict, out_path: str | None = None, timeout: float = 600):
    """Run oracle/_ref/harness_<name> (reference libponyrt). Returns the JSON
    timing line and, if out_path is given, the raw u64 output array."""
    exe = harness_path(name)
    if not os.path.exists(exe):
        raise FileNotFoundError(exe)
    cmd = [exe]
    for k, v in args.items():
        cmd += [f"--{k}", str(v)]
    if out_path:
        cmd += ["--out", out_path]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, check=True)
    line = [ln for ln in res.stdout.splitlines() if ln.startswith("{")][-1]
    info = json.loads(line)
    data = np.fromfile(out_path, dtype="<u8") if out_path else None
    return info, data
