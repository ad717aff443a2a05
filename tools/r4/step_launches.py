"""Every kernel launch of one graph-replayed train step (between two adamw_update launches) from a
rocprofv3 kernel trace, in order: start offset, duration, grid / workgroup size, VGPRs, LDS, short name.
python tools/r4/step_launches.py run_kernel_trace.csv [name-regex]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adamw_update" in r["Kernel_Name"]]
seg = rows[idx[-3] + 1:idx[-2] + 1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
t0 = int(seg[0]["Start_Timestamp"])
for r in seg:
    n = r["Kernel_Name"]
    if pat and not pat.search(n):
        continue
    m = re.search(r"::(\w+?<[^()]*>|\w+?)\(", n) or re.search(r"(\w+)", n)
    k = m.group(1) if m else n[:60]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
    w = r.get("Workgroup_Size", r.get("Workgroup_Size_X", "?"))
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  grid {g:>8} wg {w:>5} vgpr {r.get('VGPR_Count', '?'):>4} "
          f"lds {r.get('LDS_Block_Size', r.get('Lds_Size', '?')):>6} q{r.get('Queue_Id', '?')}  {k[:110]}")
