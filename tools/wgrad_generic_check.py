"""Exactness of the bf16 wgrad's GENERIC row walk (INC=false: chosen when To < rows_per_step) on
bf16-rounded inputs vs float64, several repeats -- used to test a library build (MTTS_LIB) for the
packed-fp32 fault of DESIGN.md §9 (the generic instantiation is the one whose packed-fp32 build holds
v_pk_mul_f32 ... op_sel:[0,1] op_sel_hi:[1,0])."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd")]
from matcha.models.components import _ops as O  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
worst = 0
for name, B, T, Cin, Cout, k in [("lin_T16", 1200, 16, 256, 768, 1), ("conv3_T24", 800, 24, 512, 256, 3)]:
    x = torch.randn(B, T, Cin, device=dev).bfloat16().float()
    dy = torch.randn(B, T, Cout, device=dev).bfloat16().float()
    pad = k // 2
    ref = torch.nn.grad.conv1d_weight(x.double().transpose(1, 2), (Cout, Cin, k), dy.double().transpose(1, 2), padding=pad)
    refb = dy.double().sum((0, 1))
    outs = []
    for rep in range(4):
        dw = torch.full((Cout, Cin, k), float("nan"), device=dev)
        db = torch.full((Cout,), float("nan"), device=dev)
        O._wgrad(dy, T, 1, 0, x, T, T, B, 1, [j - pad for j in range(k)], Cin, Cout, dw, (Cin * k, k, 1),
                 prec=O.PREC_BF16, db=db)
        torch.cuda.synchronize()
        outs.append(dw.clone())
        bad = ((dw.double() - ref).abs() > 1e-4 * ref.abs().max()).sum().item()
        bad_b = ((db.double() - refb).abs() > 1e-3).sum().item()
        worst = max(worst, bad + bad_b)
        print(f"{name} rep{rep}: dw bad {bad} db bad {bad_b}", flush=True)
    print("   bitwise identical:", all(torch.equal(outs[0], o) for o in outs[1:]), flush=True)
sys.exit(1 if worst else 0)
