"""The torch fp32 oracle (oracle/matcha_oracle.py) against fixtures produced by running the reference
model code (tests/golden/_decoder_golden.py).  Tolerances are fp32 reordering noise."""
from __future__ import annotations

from pathlib import Path
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from golden.weights_recipe import apply_recipe
from oracle import matcha_oracle as MO
import oracle_bind as O

GD = np.load(Path(__file__).parent / "golden" / "decoder_golden.npz")
GM = np.load(Path(__file__).parent / "golden" / "model_golden.npz")

SMALL = dict(channels=(32, 32), attention_head_dim=16, num_heads=2)
FULL = dict(channels=(256, 256), attention_head_dim=64, num_heads=4)
CASES = [("s64_", SMALL, 8, 11), ("s65_", SMALL, 8, 21), ("s33_", SMALL, 8, 31), ("f97_", FULL, 80, 12)]


def oracle_maximum_path(value: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    path, _ = O.maximum_path(value.detach().float().numpy(), mask.detach().float().numpy())
    return torch.from_numpy(path)


def build_cfm(params, n_feats, seed):
    cfm = MO.CFMOracle(2 * n_feats, n_feats, SimpleNamespace(sigma_min=1e-4), params)
    apply_recipe(cfm, seed)
    return cfm.eval()


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.mark.parametrize("prefix,params,n_feats,seed", CASES)
def test_decoder_forward_and_loss(prefix, params, n_feats, seed):
    torch.set_num_threads(8)
    cfm = build_cfm(params, n_feats, seed)
    names = [n for n, _ in cfm.named_parameters()]
    assert names == list(GD[prefix + "param_names"])  # the reference's state_dict keys
    g = lambda k: torch.from_numpy(GD[prefix + k])  # noqa: E731
    with torch.no_grad():
        u = cfm.estimator(g("phi"), g("mask"), g("mu"), g("t"))
    assert rel(u.numpy(), GD[prefix + "u"]) < 1e-5
    mu = g("mu").clone().requires_grad_(True)
    loss, phi_t = cfm.compute_loss(g("x1"), g("mask"), mu, t=g("loss_t"), z=g("loss_z"))
    loss.backward()
    assert abs(loss.item() - GD[prefix + "loss"]) <= 1e-5 * abs(GD[prefix + "loss"])
    assert rel(phi_t.detach().numpy(), GD[prefix + "phi_t"]) < 1e-6
    assert rel(mu.grad.numpy(), GD[prefix + "grad_mu"]) < 1e-4
    gn = np.array([p.grad.double().norm().item() for _, p in cfm.named_parameters()])
    np.testing.assert_allclose(gn, GD[prefix + "grad_norms"], rtol=1e-4, atol=1e-7)
    if prefix + "grad." + names[0] in GD.files:
        for n, p in cfm.named_parameters():
            ref = GD[prefix + "grad." + n]
            assert rel(p.grad.numpy(), ref) < 2e-4 or np.abs(ref).max() < 1e-7, n


def test_matcha_forward_losses_and_alignment():
    torch.set_num_threads(8)
    model = MO.MatchaTTSOracle(150, 80, 192, maximum_path=oracle_maximum_path)
    apply_recipe(model, 13)
    model.eval()
    assert [n for n, _ in model.named_parameters()] == list(GM["m_param_names"])
    enc = sum(p.numel() for p in model.encoder.parameters())
    dec = sum(p.numel() for p in model.decoder.parameters())
    assert [enc, dec] == list(GM["m_nparams"]) == [7189969, 11782992]
    g = lambda k: torch.from_numpy(GM[k])  # noqa: E731
    with torch.no_grad():
        mu_x, logw, x_mask = model.encoder(g("m_x"), g("m_x_lengths"))
    assert rel(mu_x.numpy(), GM["m_mu_x"]) < 1e-5
    assert rel(logw.numpy(), GM["m_logw"]) < 1e-5
    dur, prior, diff, attn = model(g("m_x"), g("m_x_lengths"), g("m_y"), g("m_y_lengths"), t=g("m_t"), z=g("m_z"))
    np.testing.assert_array_equal(attn.numpy().astype(np.int8), GM["m_attn"])  # MAS bit-exact
    np.testing.assert_allclose([dur.item(), prior.item(), diff.item()], GM["m_losses"], rtol=1e-5)
    (dur + prior + diff).backward()
    gn = np.array([p.grad.double().norm().item() if p.grad is not None else 0.0 for _, p in model.named_parameters()])
    np.testing.assert_allclose(gn, GM["m_grad_norms"], rtol=2e-4, atol=1e-7)
