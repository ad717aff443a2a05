"""Prints the headline fields of a bench.py JSON line (the last JSON line of the file)."""
import json
import sys

line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print("value", d["value"], "ms/step", d["ms_per_step"], "planes", d["config"].get("weight_planes"),
      "mode", (d.get("precision_check") or {}).get("run_mode"))
pc = d.get("precision_check") or {}
for k, v in (pc.get("modes") or {}).items():
    print("  precision", k, v)
for k, v in (pc.get("grads") or {}).items():
    print("  grads", k, v)
for k in ("roofline", "roofline_wgrad", "roofline_attn", "roofline_mas"):
    r = d.get(k) or {}
    print(k, {x: r.get(x) for x in ("timing", "achieved", "frac", "avg_launch_us", "traffic")})
for k, v in (d.get("extra_configs") or {}).items():
    print("extra", k, {x: v.get(x) for x in ("ms_per_step", "utterances_per_s", "losses")})
g = d.get("graph_replay_profile") or {}
print("graph", {k: g.get(k) for k in ("kernels_per_step", "step_span_us", "step_busy_us")}, g.get("families"))
print("cpu", (d.get("cpu_baseline") or {}).get("value"), "mas", d.get("maximum_path", {}).get("value"))
