"""Probe the attention kernels' fragment layouts: V = one-hot rows makes o[q, :T] = P[q, :]."""
import sys, math
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd")]
import torch
from matcha.models.components import _ops as O
torch.set_printoptions(precision=3, linewidth=200, sci_mode=False)
dev = torch.device("cuda")
T = 32
g = torch.Generator().manual_seed(0)
qkv = torch.zeros(1, T, 192)
qkv[0, :, :128] = torch.randn(T, 128, generator=g)
qkv[0, :, 128:128 + T] = torch.eye(T)
qkv = qkv.to(dev)
bias = torch.ones(1, T, device=dev)
ref = (qkv[0, :, :64] @ qkv[0, :, 64:128].T / 8 + 1).softmax(-1)
for prec in (False, True):
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=prec):
        o = O.attention_tm(qkv, bias, 1)
    P = o[0, :, :T]
    print("bf16" if prec else "fp32", "max|P-ref| =", (P - ref).abs().max().item())
    if prec:
        print("ref row0", ref[0, :16]); print("got row0", P[0, :16])
        print("ref row5", ref[5, :16]); print("got row5", P[5, :16])
        # which ref column best matches each got column
        cols = [(P[:, j:j+1] - ref).abs().sum(0).argmin().item() for j in range(T)]
        print("col map", cols)
        rows = [(P[i:i+1] - ref).abs().sum(1).argmin().item() for i in range(T)]
        print("row map", rows)
