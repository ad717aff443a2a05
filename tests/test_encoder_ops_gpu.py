"""Text-encoder operators on the GPU (train mode): RoPE against the reference formula, and every
dropout-carrying op's backward against central differences of its own forward with the dropout masks
replayed (same device RNG state -> same seeds -> same counter-based masks).  Exact-fp32 MFMA path."""
from __future__ import annotations

import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _dirderiv_check(fn, inputs, rtol=2e-3, eps=1e-3, seed=7):
    """<grad f . v> (analytic, one backward) vs (f(x+eps v) - f(x-eps v)) / 2eps for a random direction v
    over every floating input, with the op's RNG draws replayed for each evaluation."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    dirs = [torch.randn(x.shape, generator=g).to(DEV) for x in inputs]
    w = None

    def run(xs):
        torch.cuda.manual_seed(1234)
        return fn(*xs)

    xs = [x.detach().clone().requires_grad_(True) for x in inputs]
    y = run(xs)
    w = torch.randn(y.shape, generator=g).to(DEV)
    (y * w).sum().backward()
    analytic = sum((x.grad * d).sum().item() for x, d in zip(xs, dirs))
    with torch.no_grad():
        yp = run([x + eps * d for x, d in zip(inputs, dirs)])
        ym = run([x - eps * d for x, d in zip(inputs, dirs)])
        numeric = ((yp - ym) * w).sum().item() / (2 * eps)
    assert abs(analytic - numeric) <= rtol * max(abs(numeric), 1.0), (analytic, numeric)
    return y


def _mask(B, T, seed=0):
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(T // 2, T + 1, (B,), generator=g)
    lens[0] = T
    return (torch.arange(T)[None] < lens[:, None]).float().to(DEV)


@pytest.mark.parametrize("d", [96, 20])  # 96: the float4 kernel (the model's head dim); 20: the scalar one
def test_rope_matches_reference_formula(d):
    from matcha.models.components import _ops as O
    from matcha.models.components.text_encoder import RotaryPositionalEmbeddings

    B, T, H = 3, 37, 2
    qkv = torch.randn(B, T, 3 * H * d, device=DEV, requires_grad=True)
    rp = RotaryPositionalEmbeddings(d * 0.5)
    cos, sin = rp.tables(T, DEV)
    out = O.rope_tm(qkv, cos, sin, H, rp.feature_dim)
    # reference (text_encoder.py:128-143) on [B, H, T, d]
    x = qkv.detach().clone().requires_grad_(True)
    q, k, v = x.split(H * d, dim=-1)
    R, half = rp.feature_dim, rp.feature_dim // 2
    cc, ss = torch.cat([cos, cos], 1)[:, None, :], torch.cat([sin, sin], 1)[:, None, :]

    def ref(t):
        t = t.view(B, T, H, d)
        tr, tp = t[..., :R], t[..., R:]
        neg = torch.cat([-tr[..., half:], tr[..., :half]], -1)
        return torch.cat([tr * cc + neg * ss, tp], -1).reshape(B, T, H * d)

    expect = torch.cat([ref(q), ref(k), v], -1)
    torch.testing.assert_close(out, expect, rtol=1e-6, atol=1e-6)
    gout = torch.randn_like(out)
    out.backward(gout)
    expect.backward(gout)
    torch.testing.assert_close(qkv.grad, x.grad, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("relu,p", [(True, 0.1), (False, 0.1), (True, 0.0)])
def test_layer_norm_tail_grad(relu, p):
    from matcha.models.components import _ops as O

    M, C = 300, 192
    x = torch.randn(M, C, device=DEV)
    # ReLU inputs kept away from the kink (finite differences across it are meaningless): |xhat*w| < 3
    # and b = +-3 fixes the gate -- half the channels pass, half are cut
    w = (torch.rand(C, device=DEV) * 0.2 + 0.1) * torch.sign(torch.randn(C, device=DEV))
    b = torch.where(torch.arange(C, device=DEV) % 2 == 0, 3.0, -3.0)
    y = _dirderiv_check(lambda x_, w_, b_: O.layer_norm_tm(x_, w_, b_, 1e-5, relu=relu, dropout_p=p), [x, w, b])
    if p > 0 and not relu:
        frac = (y == 0).float().mean().item()
        assert abs(frac - p) < 0.02


@pytest.mark.parametrize("k", [5, 3])
def test_conv_relu_dropout_grad(k):
    from matcha.models.components import _ops as O

    B, T, Cin, Cout = 3, 50, 64, 96
    x = torch.randn(B, T, Cin, device=DEV)
    w = torch.randn(Cout, Cin, k, device=DEV) / math.sqrt(Cin * k) * 0.2  # |w.x| << 3: no ReLU kink crossing
    b = torch.where(torch.arange(Cout, device=DEV) % 2 == 0, 3.0, -3.0)
    m = _mask(B, T)
    _dirderiv_check(lambda x_, w_, b_: O.conv_tm(x_, w_, b_, mask=m, relu=True, dropout_p=0.1), [x, w, b])


def test_conv_residual_out_scale_grad():
    from matcha.models.components import _ops as O

    B, T, C = 2, 40, 64
    x = torch.randn(B, T, C, device=DEV)
    r = torch.randn(B, T, C, device=DEV)
    w = torch.randn(C, C, 1, device=DEV) / 8
    b = torch.randn(C, device=DEV)
    m = _mask(B, T, 1)
    _dirderiv_check(lambda x_, r_, w_, b_: O.conv_tm(x_, w_, b_, residual=r_, out_scale=m), [x, r, w, b])


def test_conv_ffn_grad_and_reference_eval():
    from matcha.models.components import _ops as O

    B, T, C, F_ = 3, 45, 64, 128
    x = torch.randn(B, T, C, device=DEV)
    w1 = torch.randn(F_, C, 3, device=DEV) / math.sqrt(3 * C) * 0.2  # ReLU away from its kink
    b1 = torch.where(torch.arange(F_, device=DEV) % 2 == 0, 3.0, -3.0)
    w2 = torch.randn(C, F_, 3, device=DEV) / math.sqrt(3 * F_)
    b2 = torch.randn(C, device=DEV) * 0.1
    m = _mask(B, T, 2)
    # eval semantics against the reference FFN (text_encoder.py:247-253): conv_net(x*m)*m, the inner conv
    # reading the unmasked ReLU output; plus the Encoder's residual and the row mask
    y = O.conv_ffn_tm(x, w1, b1, w2, b2, m, residual=x)
    mc = m[:, None, :]
    xc = x.transpose(1, 2)
    h = torch.relu(torch.nn.functional.conv1d(xc * mc, w1, b1, padding=1))
    f = torch.nn.functional.conv1d(h, w2, b2, padding=1) * mc
    torch.testing.assert_close(y, ((xc + f) * mc).transpose(1, 2), rtol=1e-4, atol=1e-4)
    _dirderiv_check(lambda x_, a, bb, c, d: O.conv_ffn_tm(x_, a, bb, c, d, m, residual=x_, p_in=0.1, p_out=0.19),
                    [x, w1, b1, w2, b2])


def test_attention_dropout_grad_and_rate():
    from matcha.models.components import _ops as O

    B, T, H, d = 2, 70, 2, 96
    qkv = torch.randn(B, T, 3 * H * d, device=DEV)
    m = _mask(B, T, 3)
    bias = (m - 1) * 1e4
    _dirderiv_check(lambda q: O.attention_tm(q, bias, H, dropout_p=0.1), [qkv])
    # rate: with v = one-hot key rows the output row is the dropped probability row
    qkv2 = torch.zeros(1, 64, 3 * 96, device=DEV)
    qkv2[0, :, :192] = torch.randn(64, 192, device=DEV)
    qkv2[0, :, 192:256] = torch.eye(64, device=DEV)
    o = O.attention_tm(qkv2, torch.zeros(1, 64, device=DEV), 1, dropout_p=0.25)
    frac = (o[0, :, :64] == 0).float().mean().item()
    assert abs(frac - 0.25) < 0.04


def test_linear_row_scales_grad():
    from matcha.models.components import _ops as O

    B, T, K, N_ = 2, 33, 64, 48
    x = torch.randn(B, T, K, device=DEV)
    w = torch.randn(N_, K, 1, device=DEV) / 8
    b = torch.randn(N_, device=DEV)
    r = torch.randn(B, T, N_, device=DEV)
    m = _mask(B, T, 4)
    _dirderiv_check(lambda x_, w_, b_, r_: O.linear_tm(x_, w_, b_, residual=r_, dropout_p=0.1, in_scale=m,
                                                       out_scale=m), [x, w, b, r])


def test_linear_one_channel_output_grad():
    """The duration predictor's 1-channel projection (gradient padded to 8 columns inside)."""
    from matcha.models.components import _ops as O

    B, T, K = 2, 29, 256
    x = torch.randn(B, T, K, device=DEV)
    w = torch.randn(1, K, 1, device=DEV) / 16
    b = torch.randn(1, device=DEV)
    m = _mask(B, T, 5)
    _dirderiv_check(lambda x_, w_, b_: O.linear_tm(x_, w_, b_, in_scale=m, out_scale=m), [x, w, b])


def test_rope_tables_are_fp32_under_autocast():
    """Regression: the tables are built with einsum, which a bf16 autocast region would run in bf16;
    the kernel reads fp32."""
    from matcha.models.components.text_encoder import RotaryPositionalEmbeddings

    rp = RotaryPositionalEmbeddings(48)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        cos, sin = rp.tables(20, DEV)
    assert cos.dtype == sin.dtype == torch.float32 and cos.is_contiguous() and cos.shape == (20, 24)


def test_encoder_bf16_deterministic():
    """Two bf16 forwards of the whole text encoder are bit-identical (the second served by the
    batched weight-packing plan the first one recorded)."""
    from matcha.models.matcha_tts import MatchaTTS
    from matcha.training import synthetic_batch

    torch.manual_seed(0)
    m = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV).eval()
    b = synthetic_batch(4, 20, 80, device=DEV)
    outs = []
    for _ in range(2):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            mu, logw, _ = m.encoder(b["x"], b["x_lengths"])
        outs.append((mu.clone(), logw.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("B,T,V,C", [(32, 120, 150, 192), (3, 17, 150, 192), (2, 5, 7, 40), (1, 300, 150, 1000)])
def test_embedding_fwd_bitwise_bwd_deterministic(B, T, V, C):
    """Token embedding * sqrt(C) (text_encoder.py:389): forward bitwise equal to torch's lookup and
    multiply; weight gradient within fp32 summation-order rounding of a float64 sum, and bitwise
    identical run to run (torch's own backward sums with atomics)."""
    import math

    from matcha.models.components.text_encoder import _Embedding

    g = torch.Generator().manual_seed(B * T + V)
    ids = torch.randint(0, V, (B, T), generator=g).to(DEV)
    ids[0, : min(T, 40)] = 3  # one token owning many rows
    w = torch.randn(V, C, generator=g).to(DEV).requires_grad_(True)
    dout = torch.randn(B, T, C, generator=g).to(DEV)
    s = math.sqrt(C)
    out = _Embedding.apply(ids, w, s)
    want = torch.nn.functional.embedding(ids, w.detach()) * s
    assert torch.equal(out, want)
    out.backward(dout)
    g1 = w.grad.clone()
    w.grad = None
    _Embedding.apply(ids, w, s).backward(dout)
    assert torch.equal(w.grad, g1)
    ref = torch.zeros(V, C, dtype=torch.float64, device=DEV).index_add_(0, ids.reshape(-1),
                                                                        (dout * s).reshape(-1, C).double())
    torch.testing.assert_close(g1.double(), ref, rtol=1e-5, atol=1e-4)


def test_encoder_grad_link_matches_autograd_sum():
    """Each encoder layer's output_conv residual gradient is added in the masked q|k|v projection's dgrad
    epilogue (GradLink) instead of autograd's add: same losses and gradients as with autograd summing
    them (MTTS_ENCODER_DX_LINK=0 path), fp32 mode, ragged lengths (the masked rows are where the
    (acc + g) * m identity needs g = 0)."""
    from matcha.models.components import text_encoder as TE
    from matcha.models.matcha_tts import MatchaTTS
    from matcha.training import synthetic_batch

    torch.manual_seed(3)
    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV).eval()
    b = synthetic_batch(5, 33, 80, device=DEV)
    res = []
    saved = TE._ENC_LINK
    try:
        for on in (False, True):
            TE._ENC_LINK = on
            model.zero_grad(set_to_none=True)
            mu, logw, m = model.encoder(b["x"], b["x_lengths"])
            ((mu * torch.linspace(-1, 1, mu.shape[1], device=DEV)[:, None]).sum() + logw.square().sum()).backward()
            grads = [p.grad.clone() for p in model.encoder.parameters() if p.grad is not None]
            res.append((mu.detach(), logw.detach(), grads))
    finally:
        TE._ENC_LINK = saved
    (mu0, lw0, g0), (mu1, lw1, g1) = res
    assert torch.equal(mu0, mu1) and torch.equal(lw0, lw1)
    assert len(g0) == len(g1) and len(g0) > 0
    worst = max(((a - c).norm() / c.norm().clamp_min(1e-30)).item() for a, c in zip(g1, g0))
    assert worst < 1e-5, worst


@pytest.mark.parametrize("inverse", [0, 1])
def test_rope_vector_and_scalar_kernels_bitwise(inverse):
    """The float4 RoPE kernel (16-byte aligned operands) and the scalar one (an unaligned view forces it)
    round identically -- the fp32 headline alignment is decided by ulp-level near-ties of mu_x."""
    from matcha import _native as N
    from matcha.models.components import _ops as O  # noqa: F401  (registers the symbols)
    from matcha.models.components.text_encoder import RotaryPositionalEmbeddings

    B, T, H, d = 4, 61, 2, 96
    rp = RotaryPositionalEmbeddings(d * 0.5)
    cos, sin = rp.tables(T, DEV)
    n = B * T * 3 * H * d
    x0 = torch.randn(n, device=DEV)
    outs = []
    for off in (0, 1):  # off 1: x / y not 16-byte aligned -> scalar kernel
        x = torch.empty(n + 4, device=DEV)[off: off + n]
        x.copy_(x0)
        buf = torch.empty(n + 4, device=DEV)
        y = buf[off: off + n]
        N.check(N.lib().mtts_rope_qk(x.data_ptr(), y.data_ptr(), B * T, T, H * d, H, rp.feature_dim, cos.data_ptr(),
                                     sin.data_ptr(), inverse, torch.cuda.current_stream().cuda_stream), "mtts_rope_qk")
        outs.append(y.clone())
    assert torch.equal(outs[0], outs[1])
