"""Per-step kernel-time breakdown and idle gaps from a rocprofv3 kernel trace (graph-replayed step
between two adamw_update launches): python tools/step_breakdown.py run_kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adamw_update" in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
seg = rows[a + 1:b + 1]
span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
busy = 0.0
gaps = []
end = int(seg[0]["Start_Timestamp"])
fam = collections.Counter()
cnt = collections.Counter()
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gaps.append(max(0, s - end) / 1e3)
    busy += (e - max(s, end)) / 1e3 if e > end else 0
    end = max(end, e)
    n = r["Kernel_Name"]
    m = re.search(r"::(\w+?)(<|\()", n) or re.search(r"(\w+)", n)
    k = m.group(1) if m else n[:30]
    if k in ("vectorized_elementwise_kernel", "elementwise_kernel_manual_unroll", "reduce_kernel",
             "elementwise_kernel", "unrolled_elementwise_kernel"):
        k = "torch:" + k
    fam[k] += (e - s) / 1e3
    cnt[k] += 1
print(f"kernels {len(seg)}  span {span:.0f} us  busy {busy:.0f} us  idle {span - busy:.0f} us "
      f"(gaps > 2 us: {sum(1 for g in gaps if g > 2)}, sum {sum(g for g in gaps if g > 2):.0f} us)")
for k, v in fam.most_common(30):
    print(f"  {v:8.1f} us  {cnt[k]:4d}x  {k}")
