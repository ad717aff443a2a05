"""Kernel time of ONE graph-replayed train step by kernel family, from a rocprofv3 kernel trace
(steps delimited by the optimizer's adamw_update launch).  python tools/step_families.py trace.csv"""
import collections, csv, re, sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in rows)
marks = [s for s, e, r in ev if "adamw_update" in r["Kernel_Name"]]
a, b = marks[-3], marks[-2]
agg = collections.defaultdict(list)
for s, e, r in ev:
    if a <= s < b:
        n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        agg[re.split(r"[<(]", n)[0]].append(e - s)
tot = sum(sum(v) for v in agg.values())
print(f"one step: {(b - a) / 1e3:.0f} us wall, kernel sum {tot / 1e3:.0f} us, {sum(len(v) for v in agg.values())} launches")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{sum(v) / 1e3:8.1f} us  n={len(v):4d}  avg={sum(v) / len(v) / 1e3:6.1f}  {k}")
