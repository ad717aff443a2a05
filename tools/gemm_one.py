"""Runs one bf16 conv_gemm shape with a given tile config N times eagerly (for rocprofv3 PMC passes)
and prints its graph-timed duration: python tools/gemm_one.py [shape] [cfg] [iters]."""
import sys
import math
from pathlib import Path
import torch
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd")]
from matcha.models.components import _ops as O

SHAPES = {  # B, T, Cin, Cout, k
    "conv3_full_256": (32, 600, 256, 256, 3), "lin_full_256_1024": (32, 600, 256, 1024, 1),
    "lin_full_1024_256": (32, 600, 1024, 256, 1), "lin_full_256_768": (32, 600, 256, 768, 1),
    "conv3_half_512": (32, 300, 512, 256, 3)}
name = sys.argv[1] if len(sys.argv) > 1 else "conv3_full_256"
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else -1
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
a16 = len(sys.argv) > 4 and sys.argv[4] == "bf16"  # A stored as bf16
B, T, Cin, Cout, k = SHAPES[name]
dev = torch.device("cuda")
x = torch.randn(B, T, Cin, device=dev)
m = torch.ones(B, T, device=dev)
w = torch.randn(Cout, Cin, k, device=dev) / math.sqrt(Cin * k)
Wp, Kp = O.pack_weight(w.permute(0, 2, 1).reshape(Cout, k * Cin), O.PREC_BF16)
y = torch.empty(B, T, Cout, device=dev)
offs = [j - k // 2 for j in range(k)]
x32 = x
x = x.to(torch.bfloat16) if a16 else x
f = lambda: O._gemm(x, T, T, B, 1, offs, Cin, Wp, Kp, Cout, y, T, prec=O.PREC_BF16, a_scale=m, tile_cfg=cfg,
                  binary_scale=True)
for _ in range(iters):
    f()
torch.cuda.synchronize()
ref = torch.nn.functional.conv1d(x32.transpose(1, 2), w, padding=k // 2).transpose(1, 2)
err = ((y - ref).norm() / ref.norm()).item()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20):
    f()
b.record(); torch.cuda.synchronize()
us = a.elapsed_time(b) / 20 * 1e3
print("ok", name, cfg, f"{us:.1f}us", f"{2*B*T*Cin*k*Cout/us/1e6:.0f}TF", f"rel_err={err:.2e}", flush=True)
