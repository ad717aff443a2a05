"""Long-form stress (BASELINE config 5: T_text = 512, T_mel = 4096) under test: the HIP attention at
the decoder's full and half resolution against a float64 reference, the CFM decoder (decoder.py:
293-371, flow_matching.py:106-151) at T = 4096 against the fp32 CPU oracle, and the whole train
forward at 512 x 4096 with length-bucketed (near-equal) lengths.  The reference's attention is full-T
(decoder.py:300-304, no cropping: matcha_tts.py:290-312 is disabled), so these are the reference's
own shapes."""
from __future__ import annotations

import math
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from golden.weights_recipe import apply_recipe

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def _attn_ref(qkv, bias, heads):
    B, T, C3 = qkv.shape
    C = C3 // 3
    d = C // heads
    q, k, v = (t.view(B, T, heads, d).transpose(1, 2) for t in qkv.split(C, dim=-1))
    s = q @ k.transpose(-1, -2) / math.sqrt(d) + bias[:, None, None, :]
    return (s.softmax(-1) @ v).transpose(1, 2).reshape(B, T, C)


@pytest.mark.parametrize("B,T", [(1, 4096), (2, 2048)])
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_attention_long_form(B, T, precision):
    from matcha.models.components import _ops as O

    heads, d = 4, 64
    g = torch.Generator().manual_seed(T + B)
    qkv = (torch.randn(B, T, 3 * heads * d, generator=g) * 1.5).to(DEV)
    lengths = torch.tensor([T] + [T - 37 * (i + 1) for i in range(B - 1)])  # bucketed: near-equal lengths
    bias = (torch.arange(T)[None, :] < lengths[:, None]).float().to(DEV)
    dout = torch.randn(B, T, heads * d, generator=g).to(DEV)
    x = qkv.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=precision == "bf16"):
        o = O.attention_tm(x, bias, heads)
    o.backward(dout)
    xr = qkv.double().requires_grad_(True)
    orf = _attn_ref(xr, bias.double(), heads)
    orf.backward(dout.double())
    if precision == "fp32":
        torch.testing.assert_close(o.double(), orf, rtol=1e-4, atol=2e-5)
        torch.testing.assert_close(x.grad.double(), xr.grad, rtol=1e-4, atol=5e-5)
    else:
        assert ((o.double() - orf).norm() / orf.norm()).item() < 1.5e-2
        C = heads * d
        gn = xr.grad.norm().item()
        for i, name in enumerate("qkv"):
            err = (x.grad[..., i * C:(i + 1) * C].double() - xr.grad[..., i * C:(i + 1) * C]).norm().item()
            assert err < 3e-2 * gn, name


def test_cfm_decoder_t4096_vs_oracle():
    """CFM.compute_loss + Decoder fwd/bwd at B=1, T=4096 (fp32): u and loss within 1e-4 relative of
    the CPU oracle (itself pinned to the reference fixtures), d mu within 1e-3, per-parameter gradient
    norms within 2e-3 -- the toy-shape bars of test_model_gpu.py at the long-form length."""
    from matcha.models.components.flow_matching import ConditionalFlowMatching
    from oracle import matcha_oracle as MO

    params = dict(channels=(256, 256), dropout=0.05, attention_head_dim=64, n_blocks=1, num_mid_blocks=2, num_heads=4)
    B, T, C = 1, 4096, 80
    cfm = ConditionalFlowMatching(2 * C, C, SimpleNamespace(sigma_min=1e-4), params).to(DEV)
    ref = MO.CFMOracle(2 * C, C, SimpleNamespace(sigma_min=1e-4), params)
    apply_recipe(cfm, 51)
    apply_recipe(ref, 51)
    cfm.eval()
    ref.eval()
    g = torch.Generator().manual_seed(52)
    L = 4096 - 93
    mask = (torch.arange(T)[None, None] < L).float()
    x1 = torch.randn(B, C, T, generator=g) * mask
    mu = torch.randn(B, C, T, generator=g)
    t = torch.rand(B, 1, 1, generator=g)
    z = torch.randn(B, C, T, generator=g)
    mu_r = mu.clone().requires_grad_(True)
    loss_r, _ = ref.compute_loss(x1, mask, mu_r, t=t, z=z)
    loss_r.backward()
    mu_d = mu.to(DEV).requires_grad_(True)
    loss, _ = cfm.compute_loss(x1.to(DEV), mask.to(DEV), mu_d, t=t.to(DEV), z=z.to(DEV))
    loss.backward()
    assert abs(loss.item() - loss_r.item()) <= 1e-4 * abs(loss_r.item()), (loss.item(), loss_r.item())
    assert rel(mu_d.grad.cpu().numpy(), mu_r.grad.numpy()) < 1e-3
    gr = dict(ref.named_parameters())
    for n, p in cfm.named_parameters():
        a, b = p.grad.double().norm().item(), gr[n].grad.double().norm().item()
        assert abs(a - b) <= 2e-3 * abs(b) + 1e-6, (n, a, b)


@pytest.mark.parametrize("precision", ["32-true", "bf16-mixed", "bf16-parity"])
def test_train_forward_512x4096_bucketed(precision):
    """MatchaTTS.forward at T_text=512, T_mel=4096 with bucketed lengths (every utterance of the
    batch within a few percent of the bucket length, as LengthBucketBatchSampler yields), B=8 as config 5:
    fp32 and bf16-parity -- alignment bit-exact and losses within 1e-4 of the oracle; bf16-mixed one plane
    -- the measured bounds of test_headline_gpu.py."""
    import oracle_bind as OB
    from matcha.models.matcha_tts import MatchaTTS
    from oracle import matcha_oracle as MO

    from test_headline_gpu import _agree, check_bf16, run_precision

    B, Tx, Ty = 8, 512, 4096  # config 5's per-GPU batch
    xl = torch.tensor([512, 497, 505, 489, 511, 500, 493, 508])
    yl = torch.tensor([4096, 3980, 4031, 3912, 4090, 4003, 3950, 4072])
    g = torch.Generator().manual_seed(61)
    x = torch.randint(1, 150, (B, Tx), generator=g) * (torch.arange(Tx)[None] < xl[:, None])
    y = torch.randn(B, 80, Ty, generator=g) * (torch.arange(Ty)[None, None] < yl[:, None, None])
    t = torch.rand(B, 1, 1, generator=g)
    z = torch.randn(B, 80, Ty, generator=g)

    def mp(value, mask):
        return torch.from_numpy(OB.maximum_path(value.detach().float().numpy(), mask.detach().float().numpy())[0])

    ref = MO.MatchaTTSOracle(150, 80, 192, maximum_path=mp)
    apply_recipe(ref, 62)
    ref.eval()
    with torch.no_grad():
        want = ref(x, xl, y, yl, t=t, z=z)
    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
    apply_recipe(model, 62)
    model.eval()
    d = lambda v: v.to(DEV)  # noqa: E731

    def fn():
        out = model(d(x), d(xl), d(y), d(yl), t=d(t), z=d(z))
        (out[0] + out[1] + out[2]).backward()
        return out

    dur, prior, diff, attn = run_precision(model, precision, fn)
    torch.cuda.synchronize()
    got = np.array([dur.item(), prior.item(), diff.item()])
    exp = np.array([float(v) for v in want[:3]])
    err = np.abs(got - exp) / np.abs(exp)
    agree = _agree(attn.cpu().numpy().astype(np.int8), want[3].numpy().astype(np.int8), xl.numpy(), yl.numpy())
    print(f"512x4096 {precision}: losses {got} oracle {exp} rel err {err} alignment agreement {agree:.6f}")
    if precision == "32-true":
        np.testing.assert_array_equal(attn.cpu().numpy(), want[3].numpy())
        assert (err <= 1e-4).all(), err
    else:
        check_bf16(precision, err, agree)
    assert all(p.grad is None or torch.isfinite(p.grad).all() for p in model.parameters())
