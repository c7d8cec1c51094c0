"""bench.py's roofline bookkeeping on the CPU: the traffic field comes only from
a PMC summary of this exact library AND of this bench's workload (the det /
storm summaries of scripts/gpu_evidence.sh carry the same library hash)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _write(path, **kw):
    with open(path, "w") as f:
        json.dump(kw, f)


def test_pmc_workload_from_field_and_suffix(tmp_path):
    assert bench.pmc_workload(str(tmp_path / "pmc_k_step_r09.json"), {}) == bench.BENCH_WORKLOAD
    assert bench.pmc_workload(str(tmp_path / "pmc_k_step_r09_det.json"), {}) == "det"
    assert bench.pmc_workload(str(tmp_path / "pmc_k_step_r09_storm.json"), {}) == "storm"
    assert bench.pmc_workload(str(tmp_path / "pmc_k_step_x.json"), {"workload": "storm"}) == "storm"


def test_pmc_traffic_skips_other_workloads(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    # same library hash: the general-path summaries sort after the bench's
    _write(prof / "pmc_k_step_r09.json", lib_sha16="abc", hbm_bytes_per_launch=1.0e8,
           workload=bench.BENCH_WORKLOAD)
    _write(prof / "pmc_k_step_r09_det.json", lib_sha16="abc", hbm_bytes_per_launch=8.0e8)
    _write(prof / "pmc_k_step_r09_storm.json", lib_sha16="abc", hbm_bytes_per_launch=7.0e9,
           workload="storm")
    _write(prof / "pmc_k_step_r08.json", lib_sha16="old", hbm_bytes_per_launch=2.0e8)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    v, src = bench.pmc_traffic("abc")
    assert v == 1.0e8 and src.endswith("pmc_k_step_r09.json")
    assert bench.pmc_traffic("nope") == (None, None)
    assert bench.pmc_traffic(None) == (None, None)


def test_committed_summaries_name_their_workload():
    """Every committed PMC summary resolves to one workload, and at most one
    bench-workload summary exists per library hash."""
    seen = {}
    prof = os.path.join(ROOT, "profiles")
    for f in sorted(os.listdir(prof)):
        if not (f.startswith("pmc_k_step_") and f.endswith(".json")):
            continue
        d = json.load(open(os.path.join(prof, f)))
        w = bench.pmc_workload(f, d)
        assert w in (bench.BENCH_WORKLOAD, "det", "storm"), f
        if w == bench.BENCH_WORKLOAD and d.get("lib_sha16"):
            seen.setdefault(d["lib_sha16"], []).append(f)
    dup = {k: v for k, v in seen.items() if len(v) > 1}
    assert not dup, dup
