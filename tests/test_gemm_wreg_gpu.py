"""Weight-stationary GEMM schedule (csrc/conv_gemm_wreg.hip, schedule id MTTS_GEMM_WREG): the K <= 256 linears and
1x1 convs of the decoder (FeedForward up-projection / GELU' dgrad, q|k|v and out projections, res_conv) with W held
in registers.  Every epilogue kind the kernel specialises (plain bf16 / fp32 C, GELU with the bf16 pre-activation,
GELU' on a bf16 aux, and the run-time fallback) on ragged row counts, column counts that are not a multiple of its
128-column workgroup, a 0/1 row mask, fp32 / bf16 A and one / two weight planes: bitwise equal to the
register-staged schedule 7 (fp32 A) / the LDS-DMA schedule 41 (bf16 A), which run the same MFMA order per
element, and within bf16 rounding of a float64 product."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
WREG = 96  # include/mtts_decoder.h MTTS_GEMM_WREG

KINDS = ["lin16", "lin32", "gelu", "dgelu", "runtime"]


def _case(kind, B, T, K, N, a16, split, masked, seed):
    from matcha.models.components import _ops as O

    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(B, T, K, generator=g).bfloat16().float()
    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV)
    if split:
        hi = w.bfloat16()
        Wp = torch.cat([hi, (w - hi.float()).bfloat16()]).contiguous()
        Wp._mtts_w_split = True
        Kp = K
    else:
        Wp, Kp = O.pack_weight(w, O.PREC_BF16)
    kw = dict(act=O.ACT_NONE)
    if masked:
        kw["a_scale"] = (torch.rand(B * T, generator=g) > 0.25).float().to(DEV)
    c16 = kind in ("lin16", "gelu", "dgelu")
    if kind in ("lin32", "gelu", "runtime"):
        kw["bias"] = torch.randn(N, generator=g).to(DEV)
    if kind in ("lin32", "gelu", "dgelu", "runtime"):
        kw["dropout_p"] = 0.1
        kw["seed"] = torch.tensor([1234, 567], dtype=torch.int32, device=DEV)
    if kind in ("lin32", "runtime"):
        kw["residual"] = torch.randn(B, T, N, generator=g).to(DEV)
    if kind == "lin32":
        kw["c_scale"] = (torch.rand(B * T, generator=g) > 0.1).float().to(DEV)
    if kind == "gelu":
        kw["act"] = O.ACT_GELU
        kw["C_pre"] = torch.empty(B, T, N, device=DEV, dtype=torch.bfloat16)
    if kind == "runtime":
        kw["act"] = O.ACT_GELU
        kw["C_pre"] = torch.empty(B, T, N, device=DEV)
    if kind == "dgelu":
        kw["act"] = O.ACT_DGELU
        kw["aux"] = torch.randn(B, T, N, generator=g).bfloat16().to(DEV)
    C = torch.empty(B, T, N, device=DEV, dtype=torch.bfloat16 if c16 else torch.float32)
    A = x.to(DEV).bfloat16() if a16 else x.to(DEV)
    return A, Wp, Kp, C, kw, x, w


def _run(A, Wp, Kp, C, kw, B, T, K, N, cfg):
    from matcha.models.components import _ops as O

    C.fill_(float("nan"))
    if kw.get("C_pre") is not None:
        kw["C_pre"].fill_(float("nan"))
    O._gemm(A, T, T, B, 1, [0], K, Wp, Kp, N, C, T, prec=O.PREC_BF16, tile_cfg=cfg, **kw)
    torch.cuda.synchronize()
    return C.float().clone(), (kw["C_pre"].float().clone() if kw.get("C_pre") is not None else None)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("B,T,K,N,a16,split,masked", [
    (3, 137, 256, 1024, False, False, True),   # FF up-projection shape class, ragged rows
    (2, 301, 256, 768, True, True, False),     # q|k|v, two planes, bf16 A
    (4, 77, 160, 320, True, False, True),      # K = 160, N not a multiple of 128
    (5, 40, 192, 192, False, True, True),      # the encoder's K = 192
    (1, 600, 80, 256, True, True, False),      # K = 80
])
def test_wreg_bitwise_vs_register_schedule(kind, B, T, K, N, a16, split, masked):
    A, Wp, Kp, C, kw, x, w = _case(kind, B, T, K, N, a16, split, masked, seed=B * T + K + N)
    got, got_pre = _run(A, Wp, Kp, C, kw, B, T, K, N, WREG)
    want, want_pre = _run(A, Wp, Kp, C, kw, B, T, K, N, 41 if a16 else 7)
    assert not torch.isnan(got).any()
    assert torch.equal(got, want)
    if got_pre is not None:
        assert torch.equal(got_pre, want_pre)
    if kind == "lin16":  # the product itself, against float64 (bf16-exact A, weights rounded to the planes' sum)
        wq = Wp[:N].float() + (Wp[N:].float() if split else 0.0)
        ref = x.double().reshape(-1, K) @ wq[:, :K].double().cpu().T
        if masked:
            ref *= kw["a_scale"].double().cpu()[:, None]
        err = (got.reshape(-1, N).double().cpu() - ref).abs().max().item()
        assert err <= 2 ** -8 * ref.abs().max().item() + 1e-6, err


def test_wreg_heuristic_and_unsupported_shapes():
    """On the step's FF up-projection shape the heuristic (which picks this kernel there) equals schedule 7
    bitwise; a multi-tap conv that asks for the schedule explicitly gets MTTS_ERR_UNSUPPORTED (no silent
    fallback)."""
    from matcha.models.components import _ops as O
    from matcha import _native as N

    B, T, K, Nn = 16, 600, 256, 1024
    A, Wp, Kp, C, kw, x, w = _case("gelu", B, T, K, Nn, False, False, False, seed=3)
    got, _ = _run(A, Wp, Kp, C, kw, B, T, K, Nn, -1)
    want, _ = _run(A, Wp, Kp, C, kw, B, T, K, Nn, 7)
    assert torch.equal(got, want)
    x3 = torch.randn(2, 50, 256, device=DEV)
    Wp3, Kp3 = O.pack_weight(torch.randn(128, 3 * 256, device=DEV), O.PREC_BF16)
    y = torch.empty(2, 50, 128, device=DEV)
    with pytest.raises(N.NativeError):
        O._gemm(x3, 50, 50, 2, 1, [-1, 0, 1], 256, Wp3, Kp3, 128, y, 50, prec=O.PREC_BF16, tile_cfg=WREG)


@pytest.mark.parametrize("kind", ["lin16", "lin32", "dgelu"])
def test_wreg_refuses_n_mod_8_eq_4(kind):
    """the kernel finishes 8 columns per lane, so N % 8 == 4 (here N = 196 in rows of ldc = 200) must
    not reach it: the heuristic picks another schedule (bitwise equal to schedule 41, the 4 columns past N left
    untouched) and an explicit request fails loudly."""
    from matcha import _native as N
    from matcha.models.components import _ops as O

    B, T, K, Nn, ld = 2, 150, 256, 196, 200
    A, Wp, Kp, _, kw, x, w = _case(kind, B, T, K, Nn, True, False, True, seed=5)
    for k in ("residual", "aux"):  # epilogue streams with the output's row pitch
        if k in kw:
            t = torch.zeros(B, T, ld, device=DEV, dtype=kw[k].dtype)
            t[..., :Nn] = kw[k]
            kw[k] = t
    dt = torch.bfloat16 if kind in ("lin16", "dgelu") else torch.float32
    outs = []
    for cfg in (-1, 41):
        C = torch.full((B, T, ld), float("nan"), device=DEV, dtype=dt)
        O._gemm(A, T, T, B, 1, [0], K, Wp, Kp, Nn, C, T, prec=O.PREC_BF16, tile_cfg=cfg, **kw)
        torch.cuda.synchronize()
        assert torch.isnan(C[..., Nn:].float()).all(), "columns past N written"
        outs.append(C[..., :Nn].float())
    assert torch.equal(outs[0], outs[1])
    C = torch.empty(B, T, ld, device=DEV, dtype=dt)
    with pytest.raises(N.NativeError):
        O._gemm(A, T, T, B, 1, [0], K, Wp, Kp, Nn, C, T, prec=O.PREC_BF16, tile_cfg=WREG, **kw)
