"""Summarise tools/pmc_sq.sh output: per kernel, the mean of each counter over its dispatches."""
import csv, glob, sys
from collections import defaultdict
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_sq"
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c in sorted(cs):
        v = cs[c]
        print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
