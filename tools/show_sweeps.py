import json
from collections import defaultdict
rows=[json.loads(l) for l in open("gpurun_out/sweep_panel.log") if l.startswith("{")]
print("gemm epilogue checks", [(r["cfg"], r["rel_err"]) for r in rows if "check" in r])
d=defaultdict(dict)
for r in rows:
    if "shape" in r: d[r["shape"]][r["cfg"]]=r["us"]
for s,v in d.items(): print(f"  {s:20s}", "  ".join(f"c{c}:{u:6.1f}" for c,u in v.items()))
d = defaultdict(dict); errs = []
for l in open("gpurun_out/wgrad_sweep_bf16.log"):
    if not l.startswith("{"): continue
    r = json.loads(l); d[r["shape"]][(r["kb"], r["target"], r.get("depth", 1))] = r["us"]; errs.append(max(r["rel_err"], r["db_err"]))
print("wgrad max err", max(errs))
for s, v in d.items(): print(f"  {s:20s}", "  ".join(f"{kb}/{t}/d{dp}:{u:6.1f}" for (kb, t, dp), u in v.items()))
