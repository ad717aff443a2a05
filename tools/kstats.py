"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time, per-step figures."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot/1e6:.2f} ms over {steps:g} steps = {tot/1e6/steps:.2f} ms/step, {len(rows)} kernel names")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f'{float(r["TotalDurationNs"])/1e6/steps:7.3f} ms/step {float(r["Percentage"]):5.1f}% calls/step={int(r["Calls"])/steps:6.1f} avg={float(r["AverageNs"])/1e3:8.1f}us  {r["Name"][:100]}')
