"""Workload of tools/r4/gpu_mas_pmc.sh: maximum_path on one long-form config (default 8x512x4096, lattice +
mask), a few calls, then 'ok' (tools/pmc_sq.sh checks it)."""
import runpy
import sys
from pathlib import Path

cfg = sys.argv[1] if len(sys.argv) > 1 else "8x512x4096"
sys.argv = [str(Path(__file__).resolve().parents[1] / "mas_bench.py"), "--configs", cfg, "--iters", "5"]
runpy.run_path(sys.argv[0], run_name="__main__")
print("ok")
