"""Summarise tools/pmc_traffic.sh's counters into profiles/<round>/conv_gemm_traffic.json (read by
bench.py for roofline.traffic).  FETCH_SIZE/WRITE_SIZE are in KB; FETCH_SIZE is doubled on gfx950
(MI355X_MICROARCH.md, HBM section)."""
import csv, json, sys
from pathlib import Path

src, dst = Path(sys.argv[1]), Path(sys.argv[2])


def per_dispatch(path, name):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name and "conv_gemm_kernel" in r["Kernel_Name"]:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


f = per_dispatch(src / "fetch_counter_collection.csv", "FETCH_SIZE")
w = per_dispatch(src / "write_counter_collection.csv", "WRITE_SIZE")
algo = json.load(open(src / "algorithmic.json"))
fetch_b = 2.0 * 1024 * sum(f) / len(f)
write_b = 1024 * sum(w) / len(w)
algo_b = algo["algorithmic_bytes_per_pass"] / algo["launches_per_pass"]
out = {"kernel": "conv_gemm_kernel", "workload": "one eager bf16 fwd+bwd of the bench batch (B=32, 120x600), x2 passes",
       "dispatches": len(f), "fetch_bytes_per_launch": round(fetch_b), "write_bytes_per_launch": round(write_b),
       "traffic_bytes_per_launch": round(fetch_b + write_b), "algorithmic_bytes_per_launch": round(algo_b),
       "traffic_over_algorithmic": round((fetch_b + write_b) / algo_b, 3),
       "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes, --kernel-include-regex "
                 "conv_gemm_kernel (tools/pmc_traffic.sh); KB units; FETCH_SIZE x2 on gfx950"}
dst.write_text(json.dumps(out, indent=1))
print(json.dumps(out))
