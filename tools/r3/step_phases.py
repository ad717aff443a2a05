"""Per-phase split of one graph-replayed train step from a rocprofv3 kernel trace:
encoder fwd + MAS | decoder fwd + losses | decoder bwd | encoder bwd | sums + optimizer.
python tools/r3/step_phases.py run_kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adamw_update" in r["Kernel_Name"]]
seg = rows[idx[-3] + 1:idx[-2] + 1]


def name(r):
    n = r["Kernel_Name"]
    m = re.search(r"::(\w+?)(<|\()", n) or re.search(r"(\w+)", n)
    return m.group(1) if m else n[:30]


marks = [(("mas_dp_kernel", "mas_dp_mw_kernel"), "last"), ("loss_partials_kernel", "last"), ("expand_rows_bwd_kernel", "first"),
         ("embedding_bwd_kernel", "last")]
cuts = []
for k, how in marks:
    hits = [i for i, r in enumerate(seg) if name(r) in (k if isinstance(k, tuple) else (k,))]
    cuts.append((hits[-1] if how == "last" else hits[0] - 1) + 1 if hits else None)
labels = ["encoder fwd + MAS", "decoder fwd + losses", "decoder bwd", "encoder bwd", "sums + optimizer"]
bounds = [0] + [c for c in cuts] + [len(seg)]
t0 = int(seg[0]["Start_Timestamp"])
print(f"step span {(int(seg[-1]['End_Timestamp']) - t0) / 1e3:.0f} us, {len(seg)} kernels")
for lab, a, b in zip(labels, bounds[:-1], bounds[1:]):
    if a is None or b is None or b <= a:
        print(f"{lab:24s} (marker missing)")
        continue
    part = seg[a:b]
    span = (int(part[-1]["End_Timestamp"]) - int(part[0]["Start_Timestamp"])) / 1e3
    fam = collections.Counter()
    cnt = collections.Counter()
    for r in part:
        k = name(r)
        fam[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[k] += 1
    top = ", ".join(f"{k} {v:.0f}/{cnt[k]}" for k, v in fam.most_common(6))
    print(f"{lab:24s} {span:7.0f} us  {len(part):4d} kernels  {span / len(part):5.1f} us/kernel | {top}")
