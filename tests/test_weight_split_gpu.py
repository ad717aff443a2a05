"""bf16-mixed forward GEMMs with split weight planes (MTTS_GEMM_F_W_SPLIT, csrc/pack.hip +
conv_gemm*.hip): the fp32 weights enter as hi = bf16(w) and lo = bf16(w - hi), two MFMAs per product,
so the only rounding left is the activations' (a per-sample, zero-mean error) -- the static weight
rounding was the bf16 loss error (tools/r3/precision_budget.py).  Checked against float64 on bf16-exact
activations and UNROUNDED fp32 weights, on each schedule family the forward uses: the LDS-DMA kernels
(fp32 and bf16 A, 64 x 64 and 64 x 256 tiles, split-K), the register-staged GELU schedule."""
from __future__ import annotations

import contextlib

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


@pytest.mark.parametrize("B,T,Cin,Cout,k,cfg", [(32, 120, 192, 192, 5, -1), (4, 120, 192, 576, 1, -1),
                                                (8, 120, 768, 192, 3, -1), (8, 120, 192, 768, 3, 7),
                                                (8, 120, 192, 768, 3, 12), (3, 37, 256, 80, 1, -1)])
def test_split_a_bf16x3_vs_float64(B, T, Cin, Cout, k, cfg):
    """MTTS_GEMM_F_A_SPLIT (precise_forward): fp32 activations (NOT bf16-exact) and fp32 weights, both split
    into hi + lo bf16 planes, A_hi W_hi + A_hi W_lo + A_lo W_hi -- an fp32 GEMM to ~2^-16 of the operands
    (float64 reference); the one-A-plane result (bf16 activations) is far off, so the check has teeth.  The
    text encoder's shapes (M = 32 x 120: prenet k = 5, q|k|v, FFN k = 3 both ways, mean projection) on both
    register schedules."""
    from matcha.models.components import _ops as O

    g = torch.Generator().manual_seed(B * Cout + k)
    x = torch.randn(B, T, Cin, generator=g).to(DEV)
    w = (torch.randn(Cout, Cin, k, generator=g) / (Cin * k) ** 0.5).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV)
    m = (torch.arange(T)[None] < torch.randint(T // 2, T + 1, (B,), generator=g)[:, None]).float().to(DEV)
    ref = torch.nn.functional.conv1d((x * m[..., None]).double().transpose(1, 2), w.double(), b.double(),
                                     padding=k // 2).transpose(1, 2)
    Wp, Kp = O.packed(O.spec_conv_fwd(w), O.PREC_BF16)
    assert Wp._mtts_w_split
    y = torch.empty(B, T, Cout, device=DEV)
    with O.precise_forward():
        O._gemm(x, T, T, B, 1, [j - k // 2 for j in range(k)], Cin, Wp, Kp, Cout, y, T, prec=O.PREC_BF16,
                a_scale=m, bias=b, tile_cfg=cfg)
    assert _err(y, ref) < 3e-5, _err(y, ref)
    y1 = torch.empty_like(y)  # split weights, one A plane: the activations' bf16 rounding
    O._gemm(x, T, T, B, 1, [j - k // 2 for j in range(k)], Cin, Wp, Kp, Cout, y1, T, prec=O.PREC_BF16,
            a_scale=m, bias=b, tile_cfg=cfg if cfg >= 0 else 12)
    assert _err(y1, ref) > 10 * _err(y, ref)


def test_precise_forward_encoder_backward_stays_bf16():
    """The text encoder under precise_forward: forward GEMMs bf16x3 (their outputs within ~1e-5 of the fp32
    encoder's), the backward unchanged from the bf16-mixed one (same gradients to bf16 accuracy)."""
    from golden.weights_recipe import apply_recipe
    from matcha.models.components import _ops as O
    from matcha.models.matcha_tts import MatchaTTS
    from matcha.training import synthetic_batch

    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
    apply_recipe(model, 21)
    model.eval()
    bt = synthetic_batch(8, 120, 600, seed=3, device=DEV)
    outs = {}
    for mode in ("fp32", "bf16x3", "bf16"):
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode != "fp32"), \
                (O.precise_forward() if mode == "bf16x3" else contextlib.nullcontext()):
            mu, logw, _ = model.encoder(bt["x"], bt["x_lengths"])
        (mu.square().sum() + logw.square().sum()).backward()
        outs[mode] = (mu.detach().float(), logw.detach().float(),
                      model.encoder.encoder.ffn_layers[2].conv_net[0].weight.grad.clone())
    r = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    assert r(outs["bf16x3"][0], outs["fp32"][0]) < 2e-5, r(outs["bf16x3"][0], outs["fp32"][0])
    assert r(outs["bf16x3"][1], outs["fp32"][1]) < 2e-5
    assert r(outs["bf16"][0], outs["fp32"][0]) > 10 * r(outs["bf16x3"][0], outs["fp32"][0])
    assert r(outs["bf16x3"][2], outs["fp32"][2]) < 3e-2  # bf16 backward


def test_precise_forward_fp32_encoder_equals_32true():
    """The parity policy's text encoder (precise_forward("fp32") inside the bf16 region): its forward runs
    32-true's arithmetic -- fp32 packed weights on the exact-fp32 MFMA, fp32 attention -- so mu_x and logw
    are BITWISE those of the 32-true encoder (the alignment then follows 32-true's, which matches the
    reference fixtures exactly); its backward stays the bf16 one (gradients within bf16 accuracy of the
    bf16-mixed encoder's, not equal to 32-true's)."""
    from golden.weights_recipe import apply_recipe
    from matcha.models.components import _ops as O
    from matcha.models.matcha_tts import MatchaTTS
    from matcha.training import synthetic_batch

    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
    apply_recipe(model, 22)
    model.eval()
    bt = synthetic_batch(8, 120, 600, seed=5, device=DEV)
    outs = {}
    for mode in ("32-true", "fp32fwd", "bf16"):
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode != "32-true"), \
                (O.precise_forward("fp32") if mode == "fp32fwd" else contextlib.nullcontext()):
            mu, logw, _ = model.encoder(bt["x"], bt["x_lengths"])
        (mu.square().sum() + logw.square().sum()).backward()
        outs[mode] = (mu.detach().float(), logw.detach().float(),
                      model.encoder.encoder.ffn_layers[2].conv_net[0].weight.grad.clone())
    assert torch.equal(outs["fp32fwd"][0], outs["32-true"][0])
    assert torch.equal(outs["fp32fwd"][1], outs["32-true"][1])
    r = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    assert r(outs["fp32fwd"][2], outs["32-true"][2]) < 3e-2  # bf16 backward
    assert r(outs["fp32fwd"][2], outs["bf16"][2]) < 3e-2


def test_pack_three_planes_exact():
    """MTTS_PACK_THREE_PLANES: hi = bf16(w), mid = bf16(w - hi), lo = bf16(w - hi - mid) and hi + mid + lo == w
    EXACTLY (every residual is exact in fp32 and the last one has <= 8 significant bits)."""
    from matcha.models.components import _ops as O

    g = torch.Generator().manual_seed(5)
    w = torch.randn(96, 40, generator=g).to(DEV)
    t = O._run_pack([O.spec_linear((w,))], O.PACK_BF16_SPLIT3)[0]
    assert t.shape == (3 * 96, 40) and t._mtts_w_split3
    hi, mid, lo = t[:96].float(), t[96:192].float(), t[192:].float()
    assert torch.equal(hi, w.bfloat16().float())
    assert torch.equal(mid, (w - hi).bfloat16().float())
    assert torch.equal((hi + mid) + lo, w)


@pytest.mark.parametrize("B,T,Cin,Cout,k,splits", [(32, 120, 192, 192, 5, 0), (4, 120, 192, 576, 1, 0),
                                                   (8, 120, 768, 192, 3, 0), (8, 120, 768, 192, 3, 1),
                                                   (8, 120, 192, 768, 3, 0), (3, 37, 256, 80, 1, 0),
                                                   (32, 120, 256, 1, 1, 0)])
def test_bf16x6_vs_float64(B, T, Cin, Cout, k, splits):
    """MTTS_GEMM_F_SPLIT3 (precise_forward("bf16x6")): fp32 activations and weights each as three exact bf16
    planes, the six products of combined order <= 2^-16.  Measured 1.0-2.8x the exact-fp32 MFMA kernel's
    distance to float64 (~1e-7 .. 6e-7 relative): the omitted products are ~2^-23, but the six accumulation
    chains each round -- fp32-class, not bit-faithful; bound 4x.  The text encoder's shapes
    (prenet k = 5, q|k|v, FFN k = 3 both ways with and without split-K, the mean and duration projections)."""
    from matcha.models.components import _ops as O

    g = torch.Generator().manual_seed(B * Cout + k + 7)
    x = torch.randn(B, T, Cin, generator=g).to(DEV)
    w = (torch.randn(Cout, Cin, k, generator=g) / (Cin * k) ** 0.5).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV)
    m = (torch.arange(T)[None] < torch.randint(T // 2, T + 1, (B,), generator=g)[:, None]).float().to(DEV)
    ref = torch.nn.functional.conv1d((x * m[..., None]).double().transpose(1, 2), w.double(), b.double(),
                                     padding=k // 2).transpose(1, 2)
    y = torch.empty(B, T, Cout, device=DEV)
    with O.precise_forward("bf16x6"):
        Wp, Kp = O.packed(O.spec_conv_fwd(w), O.PREC_BF16)
        assert Wp._mtts_w_split3
        O._gemm(x, T, T, B, 1, [j - k // 2 for j in range(k)], Cin, Wp, Kp, Cout, y, T, prec=O.PREC_BF16,
                a_scale=m, bias=b, splits=splits)
    Wf, Kf = O.packed(O.spec_conv_fwd(w), O.PREC_FP32)
    y32 = torch.empty_like(y)
    O._gemm(x, T, T, B, 1, [j - k // 2 for j in range(k)], Cin, Wf, Kf, Cout, y32, T, prec=O.PREC_FP32,
            a_scale=m, bias=b)
    assert _err(y, ref) < max(2e-7, 4 * _err(y32, ref)), (_err(y, ref), _err(y32, ref))


def test_precise_forward_bf16x6_encoder_close_to_32true():
    """The text encoder under precise_forward("bf16x6"): mu_x / logw within fp32 rounding of the 32-true
    encoder's (measured 2.9e-6 relative on mu_x; bound 5e-6), closer than bf16x3's, the backward bf16.  Not
    enough for the parity bar: the B=4 headline moves two durations (tests/test_headline_gpu.py)."""
    from golden.weights_recipe import apply_recipe
    from matcha.models.components import _ops as O
    from matcha.models.matcha_tts import MatchaTTS
    from matcha.training import synthetic_batch

    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
    apply_recipe(model, 23)
    model.eval()
    bt = synthetic_batch(8, 120, 600, seed=6, device=DEV)
    outs = {}
    for mode in ("32-true", "bf16x6", "bf16x3"):
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode != "32-true"), \
                (O.precise_forward(mode) if mode != "32-true" else contextlib.nullcontext()):
            mu, logw, _ = model.encoder(bt["x"], bt["x_lengths"])
        outs[mode] = (mu.float(), logw.float())
    r = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    errs = {k: (r(outs[k][0], outs["32-true"][0]), r(outs[k][1], outs["32-true"][1])) for k in ("bf16x6", "bf16x3")}
    print("encoder forward rel err vs 32-true (mu_x, logw):", errs)
    assert errs["bf16x6"][0] < 5e-6 and errs["bf16x6"][1] < 5e-6, errs
    assert errs["bf16x3"][0] > errs["bf16x6"][0], errs


@pytest.mark.parametrize("B,T,Cin,Cout,k,splits", [(32, 120, 192, 192, 5, 0), (32, 120, 768, 192, 3, 0),
                                                   (32, 120, 768, 192, 3, 4), (32, 120, 192, 576, 1, 0),
                                                   (3, 37, 256, 80, 1, 0), (32, 120, 192, 768, 3, 2)])
def test_fp32_two_steps_in_flight_bitwise(B, T, Cin, Cout, k, splits):
    """The exact-fp32 register schedules with two K steps in flight (configs 18 / 11, MTTS_GEMM_F32_DEPTH2) issue
    the same MFMAs in the same order as configs 3 / 7: bitwise equal outputs, split-K included."""
    from matcha.models.components import _ops as O

    g = torch.Generator().manual_seed(B * Cout + k + 11)
    x = torch.randn(B, T, Cin, generator=g).to(DEV)
    w = (torch.randn(Cout, Cin, k, generator=g) / (Cin * k) ** 0.5).to(DEV)
    b = torch.randn(Cout, generator=g).to(DEV)
    m = (torch.arange(T)[None] < torch.randint(T // 2, T + 1, (B,), generator=g)[:, None]).float().to(DEV)
    Wf, Kf = O.packed(O.spec_conv_fwd(w), O.PREC_FP32)
    outs = {}
    for cfg in (3, 18, 7, 11):
        y = torch.empty(B, T, Cout, device=DEV)
        O._gemm(x, T, T, B, 1, [j - k // 2 for j in range(k)], Cin, Wf, Kf, Cout, y, T, prec=O.PREC_FP32,
                a_scale=m, bias=b, tile_cfg=cfg, splits=splits)
        outs[cfg] = y
    assert torch.equal(outs[3], outs[18])
    assert torch.equal(outs[7], outs[11])
