"""HBM traffic of k_step from the rocprofv3 --pmc passes of scripts/gpu_pmc.sh.

Per step of k_step (bench.py workload): FETCH_SIZE and WRITE_SIZE (KB),
corrected as MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes — on
gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read (x2);
WRITE_SIZE is exact for 16-B-per-lane stores — and cross-checked against the
memory-side request counters (TCC_EA0_RDREQ/WRREQ x 64 B). Infinity-Cache hits
are counted by these counters, so this is an upper bound on HBM bytes.
A step of a two-pass table is two k_step launches (zone_dev.h k_step PM 1
and 2, one dispatch each per step): each kernel's mean per dispatch, summed.
Writes profiles/pmc_k_step_<tag>.json, which bench.py reports as
roofline.traffic.

usage: python scripts/pmc_traffic.py gpurun_out/pmc_<tag> <tag> [workload]
(workload: c2_message_ubench — bench.py's, the default — or det / storm)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d, tag = sys.argv[1], sys.argv[2]
workload = sys.argv[3] if len(sys.argv) > 3 else "c2_message_ubench"
vals = defaultdict(lambda: defaultdict(list))     # counter -> kernel -> values
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if "k_step" in row["Kernel_Name"]:
                vals[row["Counter_Name"]][row["Kernel_Name"]].append(float(row["Counter_Value"]))
mean = {c: sum(sum(v) / len(v) for v in per.values()) for c, per in vals.items()}
fetch_kb, write_kb = mean.get("FETCH_SIZE"), mean.get("WRITE_SIZE")
out = {
    "kernel": "k_step",
    "workload": workload,
    "dispatches": {c: {k: len(v) for k, v in per.items()} for c, per in vals.items()},
    "fetch_size_kb": fetch_kb,
    "write_size_kb": write_kb,
    "read_bytes_corrected": fetch_kb * 1024 * 2 if fetch_kb is not None else None,
    "write_bytes": write_kb * 1024 if write_kb is not None else None,
    "tcc_ea0_rdreq_bytes": mean["TCC_EA0_RDREQ_sum"] * 64 if "TCC_EA0_RDREQ_sum" in mean else None,
    "tcc_ea0_wrreq_bytes": mean["TCC_EA0_WRREQ_sum"] * 64 if "TCC_EA0_WRREQ_sum" in mean else None,
    "l2_hit_rate": (mean["TCC_HIT_sum"] / (mean["TCC_HIT_sum"] + mean["TCC_MISS_sum"])
                    if "TCC_HIT_sum" in mean else None),
    "counters_per_step": mean,
    "correction": "read = FETCH_SIZE x 1024 x 2 (gfx950 half-count on wide reads); write = WRITE_SIZE x 1024",
    "lib_sha16": (open(os.path.join(d, "lib_sha16.txt")).read().strip()
                  if os.path.exists(os.path.join(d, "lib_sha16.txt")) else None),
}
if fetch_kb is not None and write_kb is not None:
    out["hbm_bytes_per_launch"] = out["read_bytes_corrected"] + out["write_bytes"]
dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                   f"pmc_k_step_{tag}.json")
with open(dst, "w") as fh:
    json.dump(out, fh, indent=1)
print(dst, out.get("hbm_bytes_per_launch"))
