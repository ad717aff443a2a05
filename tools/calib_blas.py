"""Calibration: hipBLASLt (torch.mm, bf16 in / bf16 out) and a plain copy on the step's GEMM shapes,
graph-timed -- what the library reaches on the same M x N x K, to size the headroom of conv_gemm."""
import json, sys
from pathlib import Path
import torch
sys.path[:0] = [str(Path(__file__).resolve().parent)]
from preln_shapes import t_ev  # noqa: E402

dev = torch.device("cuda")
for M, N, K in [(19200, 768, 256), (19200, 1024, 256), (19200, 256, 1024), (19200, 256, 768), (9600, 256, 768),
                (19200, 256, 256), (9600, 256, 1536), (3840, 192, 2304)]:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    us = t_ev(lambda: torch.mm(a, w.t(), out=c))
    a32 = torch.randn(M, K, device=dev)
    c32 = torch.empty(M, N, device=dev)
    us32 = t_ev(lambda: torch.mm(a32, w.float().t(), out=c32))
    cp = torch.empty(M, N, device=dev)
    src = torch.randn(M, N, device=dev)
    uscp = t_ev(lambda: cp.copy_(src))
    print(json.dumps({"M": M, "N": N, "K": K, "blas_bf16_us": round(us, 1), "TF": round(2 * M * N * K / us / 1e6, 1),
                      "blas_fp32_us": round(us32, 1), "copy_fp32_out_us": round(uscp, 1)}), flush=True)
