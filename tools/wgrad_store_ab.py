"""Register-staged wgrad on one shape with each operand storage (fp32 / bf16 A / bf16 dY / both):
graph-timed, for rocprofv3 PMC passes too.  python tools/wgrad_store_ab.py [shape] [iters]"""
import math, sys
from pathlib import Path
import torch
sys.path[:0] = [str(Path(__file__).resolve().parent), str(Path(__file__).resolve().parent.parent / "matcha-tts-etu-upmc-ensam_amd")]
from preln_shapes import t_ev  # noqa: E402
from matcha.models.components import _ops as O  # noqa: E402

dev = torch.device("cuda")
SH = {"conv3": (32, 600, 256, 256, 3), "lin_256_1024": (32, 600, 256, 1024, 1), "lin_1024_256": (32, 600, 1024, 256, 1)}
name = sys.argv[1] if len(sys.argv) > 1 else "conv3"
B, T, Cin, Cout, k = SH[name]
x32 = torch.randn(B, T, Cin, device=dev)
dy32 = torch.randn(B, T, Cout, device=dev)
m = (torch.rand(B, T, device=dev) > 0.1).float()
pad = k // 2
dw = torch.empty(Cout, Cin, k, device=dev)
db = torch.empty(Cout, device=dev)
KB = int(sys.argv[2]) if len(sys.argv) > 2 else -1  # rows per step (-1: default 32)
TB = int(sys.argv[3]) if len(sys.argv) > 3 else -1  # target blocks
for a16, y16 in ((False, False), (True, False), (False, True), (True, True)):
    x = x32.bfloat16() if a16 else x32
    dy = dy32.bfloat16() if y16 else dy32
    run = lambda: O._wgrad(dy, T, 1, 0, x, T, T, B, 1, [j - pad for j in range(k)], Cin, Cout, dw, (Cin * k, k, 1),
                           prec=O.PREC_BF16, a_scale=m, db=db, rows_per_step=KB, target_blocks=TB,
                           depth=1 if KB > 0 else -1)
    us = t_ev(run)
    print("ok", name, f"kb={KB} tb={TB}", "A16" if a16 else "A32", "Y16" if y16 else "Y32", f"{us:.1f}us",
          f"{2 * B * T * Cin * k * Cout / us / 1e6:.0f}TF", flush=True)
