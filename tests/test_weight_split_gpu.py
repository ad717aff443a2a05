"""bf16-mixed forward GEMMs with split weight planes (MTTS_GEMM_F_W_SPLIT, csrc/pack.hip +
conv_gemm*.hip): the fp32 weights enter as hi = bf16(w) and lo = bf16(w - hi), two MFMAs per product,
so the only rounding left is the activations' (a per-sample, zero-mean error) -- the static weight
rounding was the bf16 loss error (tools/r3/precision_budget.py).  Checked against float64 on bf16-exact
activations and UNROUNDED fp32 weights, on each schedule family the forward uses: the LDS-DMA kernels
(fp32 and bf16 A, 64 x 64 and 64 x 256 tiles, split-K), the register-staged GELU schedule."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
# bf16 activations, split weights: relative error of the residual's own rounding (2^-17 of w) plus fp32
# accumulation -- about 1e-5 of the output scale; one plane (MTTS_W_SPLIT=0) gives ~3e-3
TOL = 3e-5


@pytest.fixture(autouse=True)
def _split_planes():
    from matcha.models.components import _ops as O

    old = O.set_weight_split(True)
    yield
    O.set_weight_split(old)


def _bf16_exact(*shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g).bfloat16().float().to(DEV)


def _err(got, want):
    return ((got.double() - want).abs().max() / want.abs().max()).item()


@pytest.mark.parametrize("B,T,Cin,Cout,k", [(8, 300, 256, 256, 3), (4, 77, 192, 768, 1), (2, 130, 512, 256, 1),
                                            (32, 120, 192, 192, 5), (4, 96, 80, 256, 3)])
def test_split_weight_conv_forward_vs_float64(B, T, Cin, Cout, k):
    from matcha.models.components import _ops as O

    x = _bf16_exact(B, T, Cin, seed=B + T)
    g = torch.Generator().manual_seed(Cin * k)
    w = (torch.randn(Cout, Cin, k, generator=g) / (Cin * k) ** 0.5).to(DEV)  # NOT bf16-exact
    b = torch.randn(Cout, generator=g).to(DEV)
    ref = torch.nn.functional.conv1d(x.double().transpose(1, 2), w.double(), b.double(), padding=k // 2).transpose(1, 2)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y = O.conv_tm(x, w, b, padding=k // 2)
    assert _err(y, ref) < TOL, _err(y, ref)
    # the same weights rounded to bf16 (what one plane computes) are far off: the check has teeth
    ref16 = torch.nn.functional.conv1d(x.double().transpose(1, 2), w.bfloat16().double(), b.double(),
                                       padding=k // 2).transpose(1, 2)
    assert _err(y, ref16) > 10 * TOL


@pytest.mark.parametrize("cfg", [7, 12, -1])
def test_split_weight_gelu_gemm_register_schedules(cfg):
    """The FFN's GELU projection runs the register-staged schedules (7: 32-wide K steps, 12: 64-wide, two in
    flight; -1: the heuristic's pick): split planes through the GELU epilogue against float64."""
    from matcha.models.components import _ops as O

    B, T, K, N_ = 4, 150, 256, 1024
    x = _bf16_exact(B, T, K, seed=5)
    g = torch.Generator().manual_seed(6)
    w1, b1 = (torch.randn(N_, K, generator=g) / 16).to(DEV), torch.randn(N_, generator=g).to(DEV)
    Wp = O._run_pack([O.spec_linear((w1,))], O.PACK_BF16_SPLIT)[0]
    y = torch.empty(B, T, N_, device=DEV)
    O._gemm(x, T, T, B, 1, [0], K, Wp, K, N_, y, T, prec=O.PREC_BF16, bias=b1, act=O.ACT_GELU, tile_cfg=cfg)
    ref = torch.nn.functional.gelu(x.double() @ w1.double().T + b1.double())
    assert _err(y, ref) < TOL, _err(y, ref)


def test_split_weight_packing_planes():
    """mtts_pack_weights with lo_off: hi = bf16(w), lo = bf16(w - hi)."""
    from matcha.models.components import _ops as O

    g = torch.Generator().manual_seed(9)
    w = torch.randn(96, 40, generator=g).to(DEV)
    spec = O.spec_linear((w,))
    t = O._run_pack([spec], O.PACK_BF16_SPLIT)[0]
    assert t.shape == (2 * 96, 40) and t._mtts_w_split
    hi, lo = t[:96].float(), t[96:].float()
    assert torch.equal(hi, w.bfloat16().float())
    assert torch.equal(lo, (w - hi).bfloat16().float())
    assert ((hi + lo) - w).abs().max().item() <= 2 ** -16 * w.abs().max().item()
