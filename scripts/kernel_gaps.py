"""Per-dispatch timeline of a rocprofv3 --kernel-trace CSV: for the k_step
launches of a bench run, the median duration of each launch kind and the gaps
between consecutive dispatches (the step's launch boundaries).
usage: python scripts/kernel_gaps.py <dir containing *kernel_trace.csv>"""
import csv
import glob
import os
import sys

import numpy as np

path = sys.argv[1]
files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
rows = []
for f in files:
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
ks = [r for r in rows if any(k in r[2] for k in ("k_step", "k_carry_big", "k_hot", "k_sparse"))]
def short(n):
    return n.split("(")[0].replace("void ", "")
kinds = {}
for i, (s, e, n) in enumerate(ks):
    kinds.setdefault(short(n), []).append(e - s)
for k, v in kinds.items():
    v = np.array(v[len(v) // 3:]) / 1e3          # skip the warm-up third
    print(f"{k:40s} n={len(v):4d} median {np.median(v):8.2f} us  p10 {np.percentile(v, 10):8.2f}  p90 {np.percentile(v, 90):8.2f}")
gaps = {}
for (s0, e0, n0), (s1, e1, n1) in zip(ks, ks[1:]):
    gaps.setdefault((short(n0), short(n1)), []).append(s1 - e0)
for k, v in gaps.items():
    v = np.array(v[len(v) // 3:]) / 1e3
    print(f"gap {k[0]} -> {k[1]}: n={len(v)} median {np.median(v):.2f} us p90 {np.percentile(v, 90):.2f}")
