"""Cost of the FFN GEMM epilogue pieces at 19200 x 1024 x 256 (bias / bf16 C / GELU + bf16
pre-activation / dropout / GELU' backward), per schedule, graph-timed."""
import math, sys
from pathlib import Path
import torch
sys.path[:0] = [str(Path(__file__).resolve().parent), str(Path(__file__).resolve().parent.parent / "matcha-tts-etu-upmc-ensam_amd")]
from preln_shapes import t_ev  # noqa: E402
from matcha.models.components import _ops as O  # noqa: E402

dev = torch.device("cuda")
P = O.PREC_BF16
M, K, N = 19200, 256, 1024
seed = torch.tensor([12345, 678], dtype=torch.int32, device=dev)
A32 = torch.randn(M, K, device=dev)
A16 = A32.bfloat16()
Wp, Kp = O.pack_weight(torch.randn(N, K, device=dev) / 16, P)
b = torch.randn(N, device=dev)
C32 = torch.empty(M, N, device=dev)
C16 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
aux = torch.randn(M, N, device=dev).bfloat16()
# the dgrad GEMM of the FFN backward: [M, 256] x W2^T -> [M, 1024]
Wd, Kd = O.pack_weight(torch.randn(N, K, device=dev) / 16, P)
variants = [
    ("plain_C32", dict(bias=b), C32), ("plain_C16", dict(bias=b), C16),
    ("gelu_pre_C16", dict(bias=b, act=O.ACT_GELU, C_pre=pre), C16),
    ("gelu_pre_drop_C16", dict(bias=b, act=O.ACT_GELU, C_pre=pre, dropout_p=0.05, seed=seed), C16),
    ("dgelu_C16", dict(act=O.ACT_DGELU, aux=aux), C16),
    ("dgelu_drop_C16", dict(act=O.ACT_DGELU, aux=aux, dropout_p=0.05, seed=seed), C16),
]
for a_name, A in (("A32", A32),):
    for name, kw, C in variants:
        row = []
        for cfg in (list(range(-1, 18)) + [41, 44] if a_name == "A32" else [-1, 41, 44]):
            run = lambda: O._gemm(A, M, M, 1, 1, [0], K, Wp, Kp, N, C, M, prec=P, tile_cfg=cfg, **kw)
            try:
                run(); torch.cuda.synchronize()
            except Exception as e:
                row.append(f"{cfg}:err")
                continue
            row.append(f"{cfg}:{t_ev(run):.1f}")
        print("ok", a_name, name, " ".join(row), flush=True)
