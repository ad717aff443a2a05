"""Runs one bf16 wgrad shape N times eagerly (for rocprofv3 PMC passes): python tools/wgrad_one.py [shape] [iters]."""
import sys
from pathlib import Path
import torch
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd")]
from matcha.models.components import _ops as O

SHAPES = {"lin_full_256_768": (32, 600, 256, 768, 1), "conv3_full_256": (32, 600, 256, 256, 3)}
name = sys.argv[1] if len(sys.argv) > 1 else "lin_full_256_768"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
B, T, Cin, Cout, k = SHAPES[name]
dev = torch.device("cuda")
x = torch.randn(B, T, Cin, device=dev)
dy = torch.randn(B, T, Cout, device=dev)
dw = torch.empty(Cout, Cin, k, device=dev)
db = torch.empty(Cout, device=dev)
pad = k // 2
for _ in range(iters):
    O._wgrad(dy, T, 1, 0, x, T, T, B, 1, [j - pad for j in range(k)], Cin, Cout, dw, (Cin * k, k, 1),
             prec=O.PREC_BF16, db=db)
torch.cuda.synchronize()
print("ok", name, iters)
