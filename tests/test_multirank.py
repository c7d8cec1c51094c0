"""N>1 path.  CPU: world_size 2 and 3 gloo runs of the host
plumbing (tests/mr_cpu_worker.py).  GPU: 2 ranks sharing the one GPU of the
test box through the host-staged exchange (tests/mr_worker.py) — the same
k_step outbox buckets, xout records, k_xinject landing and counter sums as the
RCCL exchange, checked bit-exact against the single-rank CPU oracle."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(script, nproc, *args, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1", f"--master-port={_port()}",
           os.path.join(HERE, script), *args]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return p.stdout


@pytest.mark.parametrize("nproc", [2, 3])
def test_host_plumbing_gloo(nproc):
    assert "MR_CPU_OK" in _launch("mr_cpu_worker.py", nproc)


TWO_RANK_CASES = ["ring", "ring1", "ubench", "ubench_det", "fanin", "gups", "storm", "fifo",
                  "fifo_seq", "spreader", "mute", "priority", "spill", "spill_one_rank",
                  "spill_one_rank_fixed", "xspill", "xspill_det", "backlog", "zones_edge",
                  "ring_prog", "det_prog"]
ZONES_4096_CASES = ["ubench_det", "storm", "spreader", "mute", "spill_one_rank", "xspill",
                    "backlog"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", TWO_RANK_CASES)
def test_two_ranks_one_gpu(case):
    out = _launch("mr_worker.py", 2, case)
    line = [l for l in out.splitlines() if l.startswith("MR_RESULT ")]
    assert line, out[-2000:]
    r = json.loads(line[-1][len("MR_RESULT "):])
    assert r["peer_write"] == int(os.environ.get("PONYC_AMD_PEER_WRITE", "0") not in ("", "0"))
    assert r["dropped"] == 0
    assert r["state_equal"]
    assert r["steps"][0] == r["steps"][1]
    assert r["delivered"][0] == r["delivered"][1]
    assert r["sent"][0] == r["sent"][1]
    assert r["pending"][0] == r["pending"][1]
    assert r["by_type"]
    assert case == "ring1" or r["remote"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", ZONES_4096_CASES)
def test_two_ranks_zones_4096(case, monkeypatch):
    """The same two-rank parity cases with 4096-actor zones forced
    (engine.hip: pick_zone_bits), as large engines run them."""
    monkeypatch.setenv("PONYC_AMD_ZONE_BITS", "12")
    test_two_ranks_one_gpu(case)


@pytest.mark.gpu
@pytest.mark.parametrize("zones", ["2048", "4096"])
@pytest.mark.parametrize("case", TWO_RANK_CASES)
def test_two_ranks_peer_write(case, zones, monkeypatch):
    """Every two-rank case with the exchange's records stored by k_step
    straight into the owner rank's inbox, mapped over IPC
    (PONYC_AMD_PEER_WRITE=1, engine.hip peer_open): only the counts go through
    the collectives. Both ranks share the test box's GPU, so the mapping is
    exercised but xGMI is not."""
    if zones == "4096":
        if case not in ZONES_4096_CASES:
            pytest.skip("the 4096-actor-zone set")
        monkeypatch.setenv("PONYC_AMD_ZONE_BITS", "12")
    monkeypatch.setenv("PONYC_AMD_PEER_WRITE", "1")
    test_two_ranks_one_gpu(case)
