"""What bf16 activation storage buys with the existing schedules: per shape, the default schedule on
fp32 A / fp32 C against every LDS-DMA schedule on bf16 A, with fp32 or bf16 C (graph-timed).
python tools/gemm_bf16_sweep.py > log"""
import json, math, sys
from pathlib import Path
import torch
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT / "tools")]
from matcha.models.components import _ops as O
from gemm_sweep2 import t_ev  # noqa: E402  (graph-timed helper)

dev = torch.device("cuda")
# name, B, T, cin, ntaps, N, residual, a_scale
SHAPES = [("dec_full_k3", 32, 600, 256, 3, 256, 0, 1), ("dec_half_k3", 32, 300, 256, 3, 256, 0, 1),
          ("ff2_full", 32, 600, 1024, 1, 256, 1, 0), ("ff2_half", 32, 300, 1024, 1, 256, 1, 0),
          ("lin_full_256_256", 32, 600, 256, 1, 256, 1, 0), ("qkv_full", 32, 600, 256, 1, 768, 0, 0),
          ("dec_full_k3_512", 32, 600, 512, 3, 256, 0, 1)]
seed = torch.tensor([12345, 678], dtype=torch.int32, device=dev)
for name, B, T, cin, k, N, res, asc in SHAPES:
    M = B * T
    x32 = torch.randn(B, T, cin, device=dev)
    x16 = x32.to(torch.bfloat16)
    w = torch.randn(N, cin * k, device=dev) / math.sqrt(cin * k)
    Wp, Kp = O.pack_weight(w, O.PREC_BF16)
    bias = torch.randn(N, device=dev)
    m = (torch.rand(M, device=dev) > 0.1).float() if asc else None
    r = torch.randn(B, T, N, device=dev) if res else None
    offs = [j - k // 2 for j in range(k)]
    for a16, c16 in [(False, False), (True, False), (True, True)]:
        x = x16 if a16 else x32
        y = torch.empty(B, T, N, device=dev, dtype=torch.bfloat16 if c16 else torch.float32)
        cands = [-1] + list(range(32, 46)) if a16 else [-1, 7, 12] + list(range(32, 46))
        best = None
        for cfg in cands:
            run = lambda: O._gemm(x, T, T, B, 1, offs, cin, Wp, Kp, N, y, T, prec=O.PREC_BF16, a_scale=m, bias=bias,
                                  residual=r, seed=seed, tile_cfg=cfg)
            try:
                run(); torch.cuda.synchronize()
            except Exception:
                continue
            us = t_ev(run)
            if best is None or us < best[1]:
                best = (cfg, us)
            if cfg == -1:
                dflt = us
        print(json.dumps({"shape": name, "A": "bf16" if a16 else "fp32", "C": "bf16" if c16 else "fp32",
                          "default_us": round(dflt, 1), "best_cfg": best[0], "best_us": round(best[1], 1),
                          "tflops_best": round(2 * M * N * cin * k / best[1] / 1e6, 1)}), flush=True)
