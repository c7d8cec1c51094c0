"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc_<tag>/p*/) per kernel:
mean counter value per dispatch of each kernel (k_step first)."""
import csv, glob, os, sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "?")
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(acc, key=lambda s: ("k_step" not in s, s)):
    print(k[:90])
    for c, v in sorted(acc[k].items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}   (n={len(v)})")
