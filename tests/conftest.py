import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_report_header(config):
    """The library every GPU test loads, by hash, at the top of each log."""
    import hashlib
    lib = os.environ.get("PONYC_AMD_LIB", os.path.join(ROOT, "ponyc_amd", "libgpuactor.so"))
    try:
        with open(lib, "rb") as f:
            sha = hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        sha = "missing"
    return f"gpu_actor library: {os.path.relpath(lib, ROOT)} sha256[:16]={sha}"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgpuactor.so)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture
def oracle():
    import pyoracle
    o = pyoracle.Oracle()
    yield o
    o.shutdown()


def make_engine(**kw):
    from ponyc_amd.engine import Engine
    return Engine(**kw)


@pytest.fixture
def engine_factory():
    """Creates engines and guarantees shutdown (the C runtime is per-process)."""
    made = []

    def make(**kw):
        e = make_engine(**kw)
        made.append(e)
        return e
    yield make
    for e in made:
        try:
            e.shutdown()
        except Exception:
            pass
