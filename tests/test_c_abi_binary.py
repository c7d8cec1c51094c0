"""A compiled C program linking -lgpuactor calls every entry point with the
prototypes a Pony program's FFI lowers to (gencall.c:
1179-1198). CPU: the prototypes agree with pony/gpu_actor/gpu_actor.pony and
include/gpu_actor.h, the struct mirrors match the header's layout (compile-time
asserts), the binary links and every call before init returns the documented
code. GPU: the same binary runs message-ubench + spreader through the FFI and
its states/counters equal the oracle's."""
import os
import re
import subprocess

import numpy as np
import pytest

from ponyc_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CDIR = os.path.join(ROOT, "tests", "c_abi")
SRC = os.path.join(CDIR, "pony_ffi_calls.c")
PONY = os.path.join(ROOT, "pony", "gpu_actor", "gpu_actor.pony")
HEADER = os.path.join(ROOT, "include", "gpu_actor.h")
LIBDIR = os.path.dirname(engine.LIB_PATH)
ROCM_LIB = "/opt/rocm/lib"

_PONY_KIND = {"I32": "i32", "U32": "u32", "U64": "u64", "F64": "f64", "None": "void"}
_C_KIND = {"int32_t": "i32", "int": "i32", "uint32_t": "u32", "uint64_t": "u64",
           "double": "f64", "void": "void"}


def _pony_kind(t: str) -> str:
    t = t.strip()
    return _PONY_KIND.get(t, "ptr")     # Pointer[A], struct/actor tags, bare lambdas


def _c_kind(t: str) -> str:
    t = re.sub(r"\b(const|struct)\b", "", t).strip()
    if "*" in t or "(" in t or t.endswith("_fn"):
        return "ptr"
    return _C_KIND[t.split()[0]]


def _split(args: str) -> list[str]:
    out, depth, cur = [], 0, ""
    for ch in args:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip() and cur.strip() != "void":
        out.append(cur)
    return out


def pony_protos() -> dict:
    src = open(PONY).read()
    out = {}
    for name, ret, args in re.findall(r"^use @(gpu_actor_\w+)\[(\w+)(?:\[.*?\])?(?: val)?\]"
                                      r"\((.*?)\)\s*$", src, re.S | re.M):
        kinds = [_pony_kind(a.split(":", 1)[1]) for a in _split(args)]
        out[name] = (_PONY_KIND.get(ret, "ptr"), kinds)
    return out


def _c_param_type(p: str) -> str:
    p = p.strip()
    if "(" in p:
        return "void (*)()"
    return re.sub(r"\s*\b\w+\s*$", "", p) if re.search(r"[\w\*]\s+\w+$", p) or "*" in p else p


def c_protos(path: str, prefix: str = "") -> dict:
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for ret, name, args in re.findall(prefix + r"^([\w\s\*]+?)\s*\b(gpu_actor_\w+)\s*\((.*?)\);",
                                      src, re.S | re.M):
        ret = ret.replace("GPU_ACTOR_API", "").strip()
        out[name] = (_c_kind(ret), [_c_kind(_c_param_type(a)) for a in _split(args)])
    return out


def test_c_prototypes_match_pony_and_header():
    pony, mine, hdr = pony_protos(), c_protos(SRC), c_protos(HEADER)
    assert len(pony) >= 23
    host_only = {"gpu_actor_set_transport", "gpu_actor_stream", "gpu_actor_last_drain_ms"}
    assert set(mine) == set(hdr), set(mine) ^ set(hdr)          # every entry point called
    assert set(hdr) - set(pony) == host_only
    for name, sig in pony.items():
        # a Pony I32 return is the header's int; U32/U64 and pointers by kind
        assert mine[name] == sig, (name, mine[name], sig)
        assert hdr[name] == sig, (name, hdr[name], sig)
    for name in host_only:
        assert mine[name] == hdr[name], name


def _build(tmp_path) -> str:
    exe = str(tmp_path / "pony_ffi_calls")
    cmd = ["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", f"-I{os.path.join(ROOT, 'include')}",
           f"-I{CDIR}", SRC, os.path.join(CDIR, "pony_layout.c"), "-o", exe,
           f"-L{LIBDIR}", "-lgpuactor", f"-Wl,-rpath,{LIBDIR}", f"-Wl,-rpath-link,{ROCM_LIB}",
           f"-Wl,-rpath,{ROCM_LIB}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_c_binary_links_and_calls_before_init(tmp_path):
    engine.load_library()          # the .so exists (fails loudly otherwise)
    exe = _build(tmp_path)
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cpu: ok" in r.stdout


COUNTS_WORDS = 7 + 16 + 1


def _counts(words: np.ndarray) -> dict:
    keys = ["steps", "delivered", "sent", "pending", "dropped", "remote", "active"]
    d = {k: int(words[i]) for i, k in enumerate(keys)}
    d["delivered_by_type"] = [int(x) for x in words[7:23]]
    return d


@pytest.mark.gpu
def test_c_binary_parity_on_gpu(tmp_path, oracle):
    from ponyc_amd import workloads as W
    exe = _build(tmp_path)
    out = str(tmp_path / "out.bin")
    r = subprocess.run([exe, "gpu", out], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    v = np.fromfile(out, dtype=np.uint64)
    steps, steps2, live, first = (int(x) for x in v[:4])
    o = 4
    c1 = _counts(v[o:o + COUNTS_WORDS]); o += COUNTS_WORDS
    c2 = _counts(v[o:o + COUNTS_WORDS]); o += COUNTS_WORDS
    ps = v[o:o + 3 * 4096].reshape(3, 4096); o += 3 * 4096
    ss = v[o:o + 5 * live].reshape(5, live); o += 5 * live
    ps2 = v[o:o + 3 * 4096].reshape(3, 4096); o += 3 * 4096
    assert o == v.size

    wu = W.ubench(oracle, 4096, 5, 20, 5489, type_id=0, mailbox_cap=16)
    ws = W.spreader(oracle, 10, type_id=1)
    so = oracle.run(0)
    co = oracle.counts()
    assert first == wu["first"]
    np.testing.assert_array_equal(ps, W.ubench_result(oracle, wu))
    np.testing.assert_array_equal(ss, W.spreader_result(oracle, ws))
    assert live == ws["nodes"]
    for k in ("delivered", "sent", "pending", "dropped", "delivered_by_type"):
        assert c1[k] == co[k], k
    assert steps == so
    for j in range(3):
        oracle.send(first + 7 * j, 0, 42)
    so2 = oracle.run(0)
    co2 = oracle.counts()
    np.testing.assert_array_equal(ps2, W.ubench_result(oracle, wu))
    for k in ("delivered", "sent", "pending", "dropped"):
        assert c2[k] == co2[k], k
    assert steps2 == so2
