"""Where the decoder FFN up-projection's time goes (19200 x 1024 x 256, fp32 A, GELU + bf16 pre-activation +
dropout, bf16 C): epilogue pieces x one / split weight planes x schedules, graph-timed.
python tools/r4/ff1_probe.py"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path[:0] = [str(ROOT / "tools"), str(ROOT / "matcha-tts-etu-upmc-ensam_amd")]
from preln_shapes import t_ev  # noqa: E402
from matcha.models.components import _ops as O  # noqa: E402

dev = torch.device("cuda")
P = O.PREC_BF16
M, K, N = 19200, 256, 1024
seed = torch.tensor([12345, 678], dtype=torch.int32, device=dev)
A = torch.randn(M, K, device=dev)
w = torch.randn(N, K, 1, device=dev) / 16
b = torch.randn(N, device=dev)
C32 = torch.empty(M, N, device=dev)
C16 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
planes = {}
for split in (False, True):
    old = O.set_weight_split(split)
    planes[split] = O.packed(O.spec_conv_fwd(w), P)
    O.set_weight_split(old)
variants = [
    ("plain_C32", dict(bias=b), C32), ("plain_C16", dict(bias=b), C16),
    ("gelu_C16", dict(bias=b, act=O.ACT_GELU), C16),
    ("gelu_pre_C16", dict(bias=b, act=O.ACT_GELU, C_pre=pre), C16),
    ("gelu_pre_drop_C16", dict(bias=b, act=O.ACT_GELU, C_pre=pre, dropout_p=0.05, seed=seed), C16),
]
for split in (False, True):
    Wp, Kp = planes[split]
    for name, kw, C in variants:
        row = []
        for cfg in [-1, 0, 1, 3, 5, 7, 12, 32, 34, 36, 38, 41, 44, 45]:
            run = lambda: O._gemm(A, M, M, 1, 1, [0], K, Wp, Kp, N, C, M, prec=P, tile_cfg=cfg, **kw)  # noqa: E731
            try:
                run()
                torch.cuda.synchronize()
            except Exception:
                row.append(f"{cfg}:err")
                continue
            row.append(f"{cfg}:{t_ev(run):.1f}")
        print("split" if split else "one", name, " ".join(row), flush=True)
