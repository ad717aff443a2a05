"""Calibration for the weight gradients: hipBLASLt dW = dY^T A (bf16 in, fp32 and bf16 out) on the
step's wgrad shapes, graph-timed."""
import json, sys
from pathlib import Path
import torch
sys.path[:0] = [str(Path(__file__).resolve().parent)]
from preln_shapes import t_ev  # noqa: E402

dev = torch.device("cuda")
for M, N, K in [(19200, 256, 768), (19200, 1024, 256), (19200, 256, 1024), (19200, 768, 256), (9600, 256, 768),
                (3840, 192, 2304)]:
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    dw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    us16 = t_ev(lambda: torch.mm(dy.t(), a, out=dw))
    dw32 = torch.empty(N, K, device=dev)
    us32 = t_ev(lambda: torch.mm(dy.t().float(), a.float(), out=dw32))
    print(json.dumps({"M(rows)": M, "N": N, "K": K, "blas_bf16_us": round(us16, 1),
                      "TF": round(2 * M * N * K / us16 / 1e6, 1), "blas_fp32_us": round(us32, 1)}), flush=True)
