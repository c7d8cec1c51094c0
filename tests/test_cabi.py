"""The drop-in boundary: libgpuactor.so loads and exports every entry point
include/gpu_actor.h declares (no compute calls: these run without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

from ponyc_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gpu_actor.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"GPU_ACTOR_API\s+[\w\s\*]+?\b(gpu_actor_\w+)\s*\(", src)))


def test_header_declarations_parsed():
    names = declared()
    assert "gpu_actor_sendv" in names and "gpu_actor_run" in names
    assert len(names) == len(engine.EXPORTS)
    assert sorted(engine.EXPORTS) == names


def test_library_exports_every_symbol():
    lib = engine.load_library()
    for name in declared():
        assert hasattr(lib, name), name


def test_exported_symbols_are_dynamic_and_default_visibility():
    out = subprocess.run(["nm", "-D", "--defined-only", engine.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    for name in declared():
        assert name in syms, name


def test_library_is_gfx950_code_object():
    # the offload bundle embeds the target id of the device code object
    blob = open(engine.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_strerror_without_gpu():
    lib = engine.load_library()
    assert lib.gpu_actor_strerror(-4) == b"mailbox overflow (messages dropped)"
    assert lib.gpu_actor_owner(7) == 0     # not initialised: a single rank


def test_calls_before_init_are_rejected():
    lib = engine.load_library()
    first = ctypes.c_uint64(0)
    assert lib.gpu_actor_type_register(0, 4, 1) == -6
    assert lib.gpu_actor_create(0, 1, ctypes.byref(first)) == -6
    assert lib.gpu_actor_send(0, 0, 0) == -6
    steps = ctypes.c_uint64(0)
    assert lib.gpu_actor_run(0, ctypes.byref(steps)) == -6


def test_engine_refuses_without_library(tmp_path, monkeypatch):
    monkeypatch.setattr(engine, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        engine.load_library(str(tmp_path / "missing.so"))


def _arity(sig: str) -> int:
    depth, n, seen = 0, 0, False
    for ch in sig:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        elif ch == "," and depth == 0:
            n += 1
        elif not ch.isspace():
            seen = True
    return n + 1 if seen and sig.strip() not in ("void",) else 0


def test_pony_package_binds_the_header():
    """pony/gpu_actor (not compilable here, ponyc needs LLVM <= 7)
    declares every entry point a Pony program uses, each with the header's
    arity, and nothing the library does not export."""
    pony = open(os.path.join(ROOT, "pony", "gpu_actor", "gpu_actor.pony")).read()
    decl = dict(re.findall(r"^use @(gpu_actor_\w+)\[.*?\]\((.*?)\)\s*$", pony, re.S | re.M))
    hdr = open(HEADER).read()
    protos = dict(re.findall(r"GPU_ACTOR_API\s+[\w\s\*]+?\b(gpu_actor_\w+)\s*\((.*?)\);", hdr, re.S))
    host_only = {"gpu_actor_set_transport", "gpu_actor_stream", "gpu_actor_last_drain_ms"}
    assert set(decl) <= set(protos)
    assert set(protos) - set(decl) == host_only
    for name, args in decl.items():
        assert _arity(args) == _arity(protos[name]), name
