"""HIP flash attention (csrc/attention.hip) against a float64 PyTorch reference of the decoder's
attention semantics: softmax(q k^T / sqrt(d) + mask[b, key]) v with the FLOAT 0/1 mask added to the
scores (transformer.py:191-370 via diffusers AttnProcessor2_0 -> F.scaled_dot_product_attention).
Forward output and the gradients of q, k, v; exact-fp32 MFMA and bf16 MFMA paths."""
from __future__ import annotations

import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _ref(qkv, bias, heads):
    B, T, C3 = qkv.shape
    C = C3 // 3
    d = C // heads
    q, k, v = (t.view(B, T, heads, d).transpose(1, 2) for t in qkv.split(C, dim=-1))
    s = q @ k.transpose(-1, -2) / math.sqrt(d) + bias[:, None, None, :]
    return (s.softmax(-1) @ v).transpose(1, 2).reshape(B, T, C)


def _case(B, T, heads, seed, d=64):
    g = torch.Generator(device="cpu").manual_seed(seed)
    qkv = torch.randn(B, T, 3 * heads * d, generator=g) * 1.5
    lengths = torch.randint(max(1, T // 2), T + 1, (B,), generator=g)
    lengths[0] = T
    bias = (torch.arange(T)[None, :] < lengths[:, None]).float()
    dout = torch.randn(B, T, heads * d, generator=g)
    return qkv.to(DEV), bias.to(DEV), dout.to(DEV)


SHAPES = [(2, 64, 4, 64), (3, 77, 4, 64), (2, 600, 4, 64), (1, 1, 4, 64), (2, 130, 2, 64), (4, 300, 4, 64),
          (1, 129, 1, 64), (2, 65, 2, 32), (2, 300, 4, 32), (3, 121, 2, 96), (1, 600, 2, 96),
          (2, 77, 2, 16), (2, 100, 1, 40),  # head dims below the compiled 32/64/96 run zero-padded
          (2, 128, 2, 96), (3, 33, 2, 96), (2, 96, 1, 64)]  # T <= 128: the short kernels' edges


@pytest.mark.parametrize("B,T,heads,d", SHAPES)
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_attention_fwd_bwd(B, T, heads, d, precision):
    from matcha.models.components import _ops as O

    qkv, bias, dout = _case(B, T, heads, seed=B * 1000 + T, d=d)
    x = qkv.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=precision == "bf16"):
        o = O.attention_tm(x, bias, heads)
    o.backward(dout)
    xr = qkv.double().requires_grad_(True)
    orf = _ref(xr, bias.double(), heads)
    orf.backward(dout.double())
    if precision == "fp32":
        # exact-fp32 products, fp32 accumulation in another order than the float64 reference
        torch.testing.assert_close(o.double(), orf, rtol=1e-4, atol=2e-5)
        torch.testing.assert_close(x.grad.double(), xr.grad, rtol=1e-4, atol=5e-5)
    else:
        rel = lambda a, b: ((a.double() - b).norm() / b.norm()).item()
        assert rel(o, orf) < 1.5e-2
        # per block, relative to the whole gradient's norm: dq = dk = 0 exactly at T = 1 (one key), where
        # bf16 rounding of dP = dO V^T against the fp32 rowsum(dO*O) leaves noise of that relative size
        C = heads * d
        gn = xr.grad.norm().item()
        for i, name in enumerate("qkv"):
            err = (x.grad[..., i * C:(i + 1) * C].double() - xr.grad[..., i * C:(i + 1) * C]).norm().item()
            assert err < 3e-2 * gn, name


def test_attention_padded_keys_are_biased_not_removed():
    """The 0/1 mask is additive: a padded key still receives exp(score)/Z weight (reference quirk)."""
    from matcha.models.components import _ops as O

    B, T, heads = 1, 40, 1
    qkv = torch.zeros(B, T, 3 * 64, device=DEV)
    qkv[0, :, 128:] = torch.arange(T, device=DEV, dtype=torch.float32)[:, None]  # v_j = j
    bias = torch.zeros(B, T, device=DEV)
    bias[0, :20] = 1.0  # keys 20..39 padded
    o = O.attention_tm(qkv, bias, heads)
    w_valid, w_pad = math.e / (20 * math.e + 20), 1.0 / (20 * math.e + 20)  # q.k = 0 everywhere
    expect = w_valid * sum(range(20)) + w_pad * sum(range(20, 40))
    torch.testing.assert_close(o[0, :, 0], torch.full((T,), expect, device=DEV), rtol=1e-5, atol=1e-5)


def test_attention_rejects_unsupported_head_dim():
    import ctypes

    from matcha import _native as N
    from matcha.models.components import _ops as O

    a = O.AttnArgs()
    buf = torch.zeros(1, 4, 3 * 128, device=DEV)
    lse = torch.zeros(1, 1, 4, device=DEV)
    o = torch.zeros(1, 4, 128, device=DEV)
    a.q = a.k = a.v = buf.data_ptr()
    a.ldq, a.o, a.ldo, a.lse = 384, o.data_ptr(), 128, lse.data_ptr()
    a.B, a.T, a.H, a.D, a.scale = 1, 4, 1, 128, 1.0
    rc = N.lib().mtts_attention_fwd(ctypes.byref(a), O.PREC_FP32, O._stream(buf))
    assert rc == -1 and b"head dim" in N.lib().mtts_last_error()


@pytest.mark.parametrize("B,T,H,D", [(4, 600, 4, 64), (3, 77, 2, 32)])
def test_attention_bf16_storage(B, T, H, D):
    """MTTS_ATTN_F_IO_BF16: bf16 q|k|v / o / dO / dq|dk|dv.  On bf16-representable inputs the forward is
    the fp32-storage kernel's output rounded once (same MFMA operands); the backward agrees to bf16
    rounding (the dO . O row sums read the rounded O)."""
    from matcha.models.components import _ops as O

    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()

    g = torch.Generator(device="cpu").manual_seed(B * T + H)
    C = H * D
    qkv = torch.randn(B, T, 3 * C, generator=g).bfloat16().float().to(DEV)
    kb = torch.zeros(B, T, device=DEV)
    for b in range(B):
        kb[b, : T - 5 * b] = 1
    do = torch.randn(B, T, C, generator=g).bfloat16().float().to(DEV)
    res = []
    for dt in (torch.float32, torch.bfloat16):
        x = qkv.to(dt)
        o = torch.empty(B, T, C, device=DEV, dtype=dt)
        lse = torch.empty(B, H, T, device=DEV)
        O._attn_fwd(x, kb, o, lse, H, O.PREC_BF16)
        dqkv = O._attn_bwd(do.to(dt), x, kb, o, lse, H, O.PREC_BF16)
        res.append((o, lse, dqkv))
    torch.cuda.synchronize()
    (o32, l32, d32), (o16, l16, d16) = res
    assert torch.equal(o16, o32.bfloat16())
    assert torch.equal(l16, l32)
    assert rel(d16.float(), d32) < 1e-2, rel(d16.float(), d32)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("B,T,H,D,p", [(32, 120, 2, 96, 0.0), (4, 120, 2, 96, 0.1), (3, 70, 4, 64, 0.0)])
def test_attention_short_path_matches_long(monkeypatch, precision, B, T, H, D, p):
    """T <= 128 runs the short kernels (a block per 32 rows, the waves split the other axis, merged in
    wave order); MTTS_ATTN_SHORT=0 sends the same call down the long kernels.  Same math in another
    summation order: fp32 agrees to 1e-5, bf16 to bf16 rounding of the products; each path is bitwise
    repeatable.  With dropout both regenerate the same mask (same (row, key) hash)."""
    from matcha.models.components import _ops as O

    g = torch.Generator(device="cpu").manual_seed(T * H + D)
    C = H * D
    qkv = torch.randn(B, T, 3 * C, generator=g).to(DEV)
    kb = torch.zeros(B, T, device=DEV)
    for b in range(B):
        kb[b, : max(1, T - 7 * b)] = 1
    do = torch.randn(B, T, C, generator=g).to(DEV)
    prec = O.PREC_FP32 if precision == "fp32" else O.PREC_BF16
    seed = torch.tensor([1234, 99], dtype=torch.int32, device=DEV) if p > 0 else None
    outs = {}
    for mode in ("1", "1", "0"):
        monkeypatch.setenv("MTTS_ATTN_SHORT", mode)
        o = torch.empty(B, T, C, device=DEV)
        lse = torch.empty(B, H, T, device=DEV)
        O._attn_fwd(qkv, kb, o, lse, H, prec, dropout_p=p, seed=seed)
        d = O._attn_bwd(do, qkv, kb, o, lse, H, prec, dropout_p=p, seed=seed)
        torch.cuda.synchronize()
        if mode in outs:
            a = outs[mode]
            assert torch.equal(a[0], o) and torch.equal(a[1], lse) and torch.equal(a[2], d)
        outs[mode] = (o, lse, d)
    (o1, l1, d1), (o0, l0, d0) = outs["1"], outs["0"]
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()
    tol = 1e-5 if precision == "fp32" else 1e-2
    assert rel(o1, o0) < tol and rel(d1, d0) < tol, (rel(o1, o0), rel(d1, d0))
    torch.testing.assert_close(l1, l0, rtol=0, atol=1e-4 if precision == "fp32" else 2e-2)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("B,T,H,D,io16", [(4, 600, 4, 64, True), (2, 300, 4, 64, False), (3, 200, 2, 96, False)])
def test_attention_bwd_merged_equals_two_launch(monkeypatch, precision, B, T, H, D, io16):
    """The merged backward (a Drow pre-pass + ONE launch whose first half runs the dQ pass and second half
    the dK/dV pass) against the two-launch sequence (MTTS_ATTN_BWD_MERGED=0): bitwise equal -- the pre-pass
    forms rowsum(dO * O) with the dQ pass's own lane mapping and summation (row_dot)."""
    from matcha.models.components import _ops as O

    if io16 and precision == "fp32":
        pytest.skip("bf16 storage needs bf16 precision")
    g = torch.Generator(device="cpu").manual_seed(B * T + D)
    C = H * D
    dt = torch.bfloat16 if io16 else torch.float32
    qkv = torch.randn(B, T, 3 * C, generator=g).to(DEV).to(dt)
    kb = torch.zeros(B, T, device=DEV)
    for b in range(B):
        kb[b, : T - 9 * b] = 1
    do = torch.randn(B, T, C, generator=g).to(DEV).to(dt)
    prec = O.PREC_FP32 if precision == "fp32" else O.PREC_BF16
    o = torch.empty(B, T, C, device=DEV, dtype=dt)
    lse = torch.empty(B, H, T, device=DEV)
    O._attn_fwd(qkv, kb, o, lse, H, prec)
    res = []
    for merged in ("1", "0"):
        monkeypatch.setenv("MTTS_ATTN_BWD_MERGED", merged)
        res.append(O._attn_bwd(do, qkv, kb, o, lse, H, prec))
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[1])
