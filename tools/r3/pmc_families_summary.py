"""tools/r3/pmc_families.sh's counters -> profiles/<round>/{gemm,wgrad,attn}_traffic.json (read by bench.py
for each roofline line's `traffic`).  FETCH_SIZE / WRITE_SIZE are in KB; FETCH_SIZE doubled on gfx950
(MI355X_MICROARCH.md, HBM section); per launch = per mtts_conv_gemm / mtts_conv_wgrad / mtts_attention_* call
(split-K combines, slab reduces and the second backward kernel counted with their call).
    python tools/r3/pmc_families_summary.py <gpurun_out dir> <profiles dir>"""
import csv
import json
import sys
from pathlib import Path

from pmc_regex import REGEX  # noqa: E402  (tools/r3/pmc_regex.py)

src, dst = Path(sys.argv[1]), Path(sys.argv[2])
only = sys.argv[3:] or ["gemm", "wgrad", "attn"]  # family names (default: the step families)
algo = json.loads((src / "algo.json").read_text())
dst.mkdir(parents=True, exist_ok=True)
for fam, rx in REGEX.items():
    if only and fam not in only:
        continue
    tot = {}
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        files = sorted((src / f"{fam}_{sub}").rglob("*counter_collection.csv"))
        vals = {}
        for r in csv.DictReader(open(files[0])):
            if r["Counter_Name"] == counter:
                d = int(r["Dispatch_Id"])
                vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
        # the profiled program also runs the warm-up pass (same dispatches as each logged pass): drop it
        ids = sorted(vals)
        warm = len(ids) * algo.get("warmup_passes", 1) // (algo["passes"] + algo.get("warmup_passes", 1))
        tot[counter] = (sum(vals[d] for d in ids[warm:]), len(ids) - warm)
    n = algo[fam]["launches"]
    fetch_b = 2.0 * 1024 * tot["FETCH_SIZE"][0] / n
    write_b = 1024 * tot["WRITE_SIZE"][0] / n
    algo_b = algo[fam]["algorithmic_bytes"] / n
    out = {"family": fam, "kernels_regex": rx,
           "workload": ("tools/r5/pmc_mas.py: two maximum_path calls on the bench batch's lattice (B=32, 120x600)"
                        if fam == "mas" else
                        f"tools/r3/pmc_families.py: two eager {algo.get('precision', 'bf16-mixed')} fwd+bwd passes of "
                        "the bench batch (B=32, 120x600)"),
           "launches": n, "dispatches": tot["FETCH_SIZE"][1], "warmup_dispatches_dropped": True, "fetch_bytes_per_launch": round(fetch_b),
           "write_bytes_per_launch": round(write_b), "traffic_bytes_per_launch": round(fetch_b + write_b),
           "algorithmic_bytes_per_launch": round(algo_b), "traffic_over_algorithmic": round((fetch_b + write_b) / algo_b, 3),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes with --kernel-include-regex; "
                     "KB units; FETCH_SIZE x2 on gfx950"}
    suffix = "_parity" if algo.get("precision") == "bf16-parity" else ""
    (dst / f"{fam}_traffic{suffix}.json").write_text(json.dumps(out, indent=1))
    print(json.dumps(out))
