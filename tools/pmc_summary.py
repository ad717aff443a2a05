"""Summarise tools/pmc_traffic.sh's counters into profiles/<round>/conv_gemm_traffic.json (read by
bench.py for roofline.traffic).  FETCH_SIZE/WRITE_SIZE are in KB; FETCH_SIZE is doubled on gfx950
(MI355X_MICROARCH.md, HBM section)."""
import csv, json, sys
from pathlib import Path

src, dst = Path(sys.argv[1]), Path(sys.argv[2])


def per_dispatch(path, name):
    vals = {}
    if not path.exists():  # rocprofv3 layout: <pass dir>/**/run_counter_collection.csv
        cands = sorted(path.parent.glob(("fetch" if name == "FETCH_SIZE" else "write") + "/**/*counter_collection.csv"))
        path = cands[0]
    for r in csv.DictReader(open(path)):
        kn = r["Kernel_Name"]
        if r["Counter_Name"] == name and ("conv_gemm_kernel" in kn or "conv_gemm_glds_kernel" in kn
                                          or "splitk_epilogue_kernel" in kn):
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


f = per_dispatch(src / "fetch_counter_collection.csv", "FETCH_SIZE")
w = per_dispatch(src / "write_counter_collection.csv", "WRITE_SIZE")
algo = json.load(open(src / "algorithmic.json" if (src / "algorithmic.json").exists() else src / "algo.json"))
# per GEMM launch (one mtts_conv_gemm call: one dispatch, or two with split-K) over the two passes
nl = algo["launches_per_pass"] * algo.get("passes", 2)
fetch_b = 2.0 * 1024 * sum(f) / nl
write_b = 1024 * sum(w) / nl
algo_b = algo["algorithmic_bytes_per_pass"] / algo["launches_per_pass"]
out = {"kernel": "conv_gemm_kernel + conv_gemm_glds_kernel (+ splitk_epilogue_kernel)", "workload": "one eager bf16 fwd+bwd of the bench batch (B=32, 120x600), x2 passes",
       "dispatches": len(f), "fetch_bytes_per_launch": round(fetch_b), "write_bytes_per_launch": round(write_b),
       "traffic_bytes_per_launch": round(fetch_b + write_b), "algorithmic_bytes_per_launch": round(algo_b),
       "traffic_over_algorithmic": round((fetch_b + write_b) / algo_b, 3),
       "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes, --kernel-include-regex "
                 "'conv_gemm_kernel|conv_gemm_glds_kernel|splitk_epilogue_kernel' (tools/pmc_traffic.sh); KB units; "
                 "FETCH_SIZE x2 on gfx950; per mtts_conv_gemm call"}
dst.write_text(json.dumps(out, indent=1))
print(json.dumps(out))
