"""Per-kernel means of tools/r5/pmc_gemm.sh's counter passes.  python tools/r5/pmc_gemm_summary.py gpurun_out/TAG"""
import collections
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
agg = collections.defaultdict(lambda: collections.defaultdict(dict))
for f in sorted(d.glob("pass*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "gemm" not in r["Kernel_Name"]:
            continue
        import re
        k = re.search(r"conv_gemm(?:_\w+)?_kernel<[^>]*>", r["Kernel_Name"]).group(0)
        key = (f.parent.name, r["Dispatch_Id"])
        agg[k][r["Counter_Name"]][key] = agg[k][r["Counter_Name"]].get(key, 0.0) + float(r["Counter_Value"])
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        vals = list(v.values())
        print(f"   {c:32s} n={len(vals):3d} mean={sum(vals) / len(vals):.4g}")
