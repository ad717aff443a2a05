"""Per-kernel PMC totals from rocprofv3 --pmc csv dirs: python tools/pmc_kernels.py dir1 [dir2 ...] [--filter s]"""
import collections
import csv
import glob
import sys

args = sys.argv[1:]
flt = ""
if "--filter" in args:
    k = args.index("--filter")
    flt = args[k + 1]
    args = args[:k] + args[k + 2:]
agg = collections.defaultdict(dict)
calls = collections.Counter()
for d in args:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if flt not in n:
                continue
            key = (n, r["Counter_Name"])
            agg[n][r["Counter_Name"]] = agg[n].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if (r.get("Dispatch_Id"), n) not in seen:
                seen.add((r.get("Dispatch_Id"), n))
        for n in {x[1] for x in seen}:
            calls[n] = max(calls[n], sum(1 for x in seen if x[1] == n))
for n, c in agg.items():
    k = max(calls[n], 1)
    print(f"{n[:80]}  ({k} dispatches, per dispatch)")
    print("   " + "  ".join(f"{a}={v / k / 1e3:.1f}k" for a, v in sorted(c.items())))
