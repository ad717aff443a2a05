"""CFM step prologue/epilogue kernels (csrc/cfm_prep.hip, csrc/losses.hip) against plain torch fp32
restatements of the reference expressions:
  phi_t + channel pack   flow_matching.py:138, decoder.py:288   (bit-exact: same fp32 op order)
  SinusoidalPosEmb       decoder.py:8-31                        (device libm sin/cos/exp: 2 ulp-ish)
  CFM + prior losses     flow_matching.py:145-149, matcha_tts.py:319-323 (fp32 reduction order differs)
"""
from __future__ import annotations

import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _inputs(B, C, T, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g, device=DEV)  # noqa: E731
    return r(B, C, T), r(B, C, T), torch.rand(B, 1, 1, generator=g, device=DEV), r(B, C, T)


@pytest.mark.parametrize("B,C,T", [(1, 80, 1), (3, 80, 63), (4, 80, 64), (2, 80, 257), (5, 128, 130), (2, 7, 65)])
def test_cfm_pack_bitwise(B, C, T):
    from matcha.models.components.flow_matching import _CfmPack

    x1, z, t, mu = _inputs(B, C, T, B * 1000 + T)
    mu.requires_grad_(True)
    s = 1e-4
    packed = _CfmPack.apply(x1, z, t, mu, s)
    phi = (1 - (1 - s) * t) * z + t * x1  # flow_matching.py:138
    want = torch.cat([phi, mu.detach()], dim=1).transpose(1, 2)  # decoder.py:288 (token-major)
    assert packed.shape == (B, T, 2 * C)
    assert torch.equal(packed, want)
    g = torch.randn_like(packed)
    packed.backward(g)
    assert torch.equal(mu.grad, g[..., C:].transpose(1, 2))


def test_cfm_pack_refuses_bad_shapes():
    from matcha.models.components.flow_matching import _CfmPack

    x1, z, t, mu = _inputs(2, 80, 16, 0)
    with pytest.raises(ValueError):
        _CfmPack.apply(x1, z[:, :40], t, mu, 1e-4)
    with pytest.raises(Exception):
        _CfmPack.apply(*(torch.randn(1, 200, 8, device=DEV) for _ in range(2)), t[:1], torch.randn(1, 200, 8,
                                                                                                   device=DEV), 1e-4)


@pytest.mark.parametrize("B,dim,scale", [(1, 80, 1000), (7, 80, 1000), (4, 256, 1), (3, 320, 1000)])
def test_time_embedding(B, dim, scale):
    from matcha.models.components.decoder import SinusoidalPosEmb

    t = torch.rand(B, device=DEV)
    got = SinusoidalPosEmb(dim)(t, scale=scale)
    half = dim // 2
    step = math.log(10000) / (half - 1)  # decoder.py:24-29
    freq = torch.exp(torch.arange(half, device=DEV).float() * -step)
    arg = scale * t.unsqueeze(1) * freq.unsqueeze(0)
    want = torch.cat((arg.sin(), arg.cos()), dim=-1)
    assert got.shape == want.shape
    # args reach ~1000 rad: a one-ulp difference in freq moves sin/cos by ~1e-4
    assert (got - want).abs().max().item() < 5e-4
    assert torch.allclose(got[:, :4], want[:, :4], atol=1e-6)


@pytest.mark.parametrize("B,C,T", [(2, 80, 50), (4, 80, 301), (3, 128, 97)])
def test_fused_losses_match_torch(B, C, T):
    from matcha.models.components.flow_matching import fused_losses

    x1, z, t, mu_y = _inputs(B, C, T, 7)
    lengths = torch.randint(1, T + 1, (B,), device=DEV)
    lengths[0] = T
    mask = (torch.arange(T, device=DEV)[None] < lengths[:, None]).float().unsqueeze(1)
    s = 1e-4
    u_pred = torch.randn(B, T, C, device=DEV, requires_grad=True)
    mu_y.requires_grad_(True)
    diff, prior = fused_losses(u_pred, mu_y, x1, z, mask, s)

    u_ref = u_pred.detach().clone().requires_grad_(True)
    mu_ref = mu_y.detach().clone().requires_grad_(True)
    u = x1 - (1 - s) * z  # flow_matching.py:141
    diff_w = torch.sum((u_ref.transpose(1, 2) - u) ** 2) / (torch.sum(mask) * C)  # :145-149, unmasked mse
    prior_w = torch.sum(0.5 * ((x1 - mu_ref) ** 2 + math.log(2 * math.pi)) * mask) / (torch.sum(mask) * C)
    torch.testing.assert_close(diff, diff_w, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(prior, prior_w, rtol=1e-5, atol=1e-6)
    (diff + 0.5 * prior).backward()
    (diff_w + 0.5 * prior_w).backward()
    torch.testing.assert_close(u_pred.grad, u_ref.grad, rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(mu_y.grad, mu_ref.grad, rtol=1e-5, atol=1e-8)


def test_fused_prior_loss_only():
    """prior_loss without the CFM term (u_pred=None, MatchaTTS with a decoder computing its own loss):
    matcha_tts.py:319-323 on the [B, T] mask."""
    from matcha.models.components.flow_matching import fused_losses

    B, C, T = 3, 80, 77
    x1, z, t, mu_y = _inputs(B, C, T, 9)
    lengths = torch.tensor([77, 40, 12], device=DEV)
    mask = (torch.arange(T, device=DEV)[None] < lengths[:, None]).float().unsqueeze(1)
    mu_y.requires_grad_(True)
    diff, prior = fused_losses(None, mu_y, x1, z, mask, 1e-4)
    mu_ref = mu_y.detach().clone().requires_grad_(True)
    prior_w = torch.sum(0.5 * ((x1 - mu_ref) ** 2 + math.log(2 * math.pi)) * mask) / (torch.sum(mask) * C)
    assert diff.item() == 0.0
    torch.testing.assert_close(prior, prior_w, rtol=1e-5, atol=1e-6)
    prior.backward()
    prior_w.backward()
    torch.testing.assert_close(mu_y.grad, mu_ref.grad, rtol=1e-5, atol=1e-8)
