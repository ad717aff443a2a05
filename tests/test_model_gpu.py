"""Product model on the MI355X against the reference fixtures (decoder_golden.npz, model_golden.npz)
and the CPU oracle.  fp32 path: loss within 1e-4 relative (the north star's bar), outputs/grads within
the tolerances written below; alignment bit-exact."""
from __future__ import annotations

from pathlib import Path
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from golden.weights_recipe import apply_recipe

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
GD = np.load(Path(__file__).parent / "golden" / "decoder_golden.npz")
GM = np.load(Path(__file__).parent / "golden" / "model_golden.npz")
SMALL = dict(channels=(32, 32), attention_head_dim=16, num_heads=2)
FULL = dict(channels=(256, 256), attention_head_dim=64, num_heads=4)
CASES = [("s64_", SMALL, 8, 11), ("s65_", SMALL, 8, 21), ("s33_", SMALL, 8, 31), ("f97_", FULL, 80, 12)]


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.mark.parametrize("prefix,params,n_feats,seed", CASES)
def test_cfm_decoder_vs_reference(prefix, params, n_feats, seed):
    from matcha.models.components.flow_matching import ConditionalFlowMatching

    cfm = ConditionalFlowMatching(2 * n_feats, n_feats, SimpleNamespace(sigma_min=1e-4), params).to(DEV)
    apply_recipe(cfm, seed)
    cfm.eval()
    g = lambda k: torch.from_numpy(GD[prefix + k]).to(DEV)  # noqa: E731
    with torch.no_grad():
        u = cfm.estimator(g("phi"), g("mask"), g("mu"), g("t"))
    assert rel(u.cpu().numpy(), GD[prefix + "u"]) < 1e-4
    mu = g("mu").clone().requires_grad_(True)
    loss, phi_t = cfm.compute_loss(g("x1"), g("mask"), mu, t=g("loss_t"), z=g("loss_z"))
    loss.backward()
    ref = float(GD[prefix + "loss"])
    assert abs(loss.item() - ref) <= 1e-4 * abs(ref)  # north star: loss within 1e-4 relative
    assert rel(mu.grad.cpu().numpy(), GD[prefix + "grad_mu"]) < 1e-3
    gn = np.array([p.grad.double().norm().item() for _, p in cfm.named_parameters()])
    np.testing.assert_allclose(gn, GD[prefix + "grad_norms"], rtol=2e-3, atol=1e-6)


def test_matcha_train_forward_vs_reference():
    from matcha.models.matcha_tts import MatchaTTS

    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
    apply_recipe(model, 13)
    model.eval()
    g = lambda k: torch.from_numpy(GM[k]).to(DEV)  # noqa: E731
    dur, prior, diff, attn = model(g("m_x"), g("m_x_lengths"), g("m_y"), g("m_y_lengths"), t=g("m_t"), z=g("m_z"))
    np.testing.assert_array_equal(attn.cpu().numpy().astype(np.int8), GM["m_attn"])
    got = np.array([dur.item(), prior.item(), diff.item()])
    np.testing.assert_allclose(got, GM["m_losses"], rtol=1e-4)
    (dur + prior + diff).backward()
    gn = np.array([p.grad.double().norm().item() if p.grad is not None else 0.0 for _, p in model.named_parameters()])
    np.testing.assert_allclose(gn, GM["m_grad_norms"], rtol=5e-3, atol=1e-6)


def test_train_step_bench_shape_vs_oracle_alignment():
    """At the bench shape (B=32, 120x600) the GPU step's alignment equals the oracle's on the same
    fp32 lattice, and one optimizer step runs with finite gradients."""
    import oracle_bind as OB
    from matcha.models.matcha_tts import MatchaTTS
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    torch.manual_seed(0)
    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
    b = synthetic_batch(32, 120, 600, device=DEV)
    model.eval()
    with torch.no_grad():
        mu_x, _, x_mask = model.encoder(b["x"], b["x_lengths"])
        lp = model.log_prior(mu_x, b["y"])
        from matcha.utils.model import sequence_mask
        y_mask = sequence_mask(b["y_lengths"], 600).unsqueeze(1).float()
        am = (x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)).squeeze(1)
        from matcha.utils.monotonic_align import maximum_path
        path = maximum_path(lp, am)
    exp, _ = OB.maximum_path(lp.cpu().numpy(), am.cpu().numpy())
    np.testing.assert_array_equal(path.cpu().numpy(), exp)
    model.train()
    tr = Trainer(model, TrainConfig())
    losses = tr.step([b])
    assert torch.isfinite(losses).all()


@pytest.mark.parametrize("length_scale,n_steps", [(1.0, 3), (3.0, 5)])
def test_synthesise_vs_oracle(length_scale, n_steps):
    """Inference: MatchaTTS.synthesise (matcha_tts.py:179-245) -- encoder, ceil'd
    durations, generate_path, attn^T mu_x, Euler ODE over the HIP decoder (flow_matching.py:42-104) --
    against the CPU oracle with the same weights and the same injected noise: identical lengths and
    alignment, mel within 1e-4 relative (fp32 MFMA mode)."""
    from matcha.models.matcha_tts import MatchaTTS
    from oracle import matcha_oracle as MO

    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
    apply_recipe(model, 17)
    model.eval()
    ref = MO.MatchaTTSOracle(150, 80, 192)
    apply_recipe(ref, 17)
    ref.eval()
    g = torch.Generator().manual_seed(3)
    B, Tx = 2, 11
    xl = torch.tensor([11, 8])
    x = torch.randint(1, 150, (B, Tx), generator=g) * (torch.arange(Tx)[None] < xl[:, None])
    with torch.no_grad():
        _, logw, x_mask = ref.encoder(x, xl)
        yl = torch.clamp_min(torch.sum(torch.ceil(torch.exp(logw) * x_mask) * length_scale, [1, 2]), 1).long()
    z = torch.randn(B, 80, MO.fix_len_compatibility(yl.max()), generator=g)
    out = model.synthesise(x.to(DEV), xl.to(DEV), n_steps, length_scale=length_scale, z=z.to(DEV))
    exp = ref.synthesise(x, xl, n_steps, length_scale=length_scale, z=z)
    np.testing.assert_array_equal(out["mel_lengths"].cpu().numpy(), exp["mel_lengths"].numpy())
    np.testing.assert_array_equal(out["attn"].cpu().numpy(), exp["attn"].numpy())
    assert rel(out["encoder_outputs"].cpu().numpy(), exp["encoder_outputs"].numpy()) < 1e-5
    assert rel(out["decoder_outputs"].cpu().numpy(), exp["decoder_outputs"].numpy()) < 1e-4
    assert rel(out["mel"].cpu().numpy(), exp["mel"].numpy()) < 1e-4


GS = np.load(Path(__file__).parent / "golden" / "synth_golden.npz")


@pytest.mark.parametrize("prefix,seed", [("a_", 23), ("b_", 29)])
def test_synthesise_vs_reference(prefix, seed):
    """MatchaTTS.synthesise against the REFERENCE's own synthesise (matcha_tts.py:178-245,
    flow_matching.py:42-104, model.py:77-114) run from a seed, with its z = randn_like(mu) * temperature
    replayed (synth_golden.npz, tests/golden/_decoder_golden.py synth_case): lengths and alignment
    exact, outputs within 1e-4 relative (fp32 MFMA mode)."""
    from matcha.models.matcha_tts import MatchaTTS

    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
    apply_recipe(model, seed)
    model.eval()
    n_steps, length_scale, temperature = GS[prefix + "cfg"]
    g = lambda k: torch.from_numpy(GS[prefix + k]).to(DEV)  # noqa: E731
    out = model.synthesise(g("x"), g("x_lengths"), int(n_steps), temperature=float(temperature),
                           length_scale=float(length_scale), z=g("z"))
    np.testing.assert_array_equal(out["mel_lengths"].cpu().numpy(), GS[prefix + "mel_lengths"])
    np.testing.assert_array_equal(out["attn"].cpu().numpy().astype(np.int8), GS[prefix + "attn"])
    for k in ("encoder_outputs", "decoder_outputs", "mel"):
        assert out[k].shape == GS[prefix + k].shape, k
        assert rel(out[k].cpu().numpy(), GS[prefix + k]) < 1e-4, k


def test_matcha_gradients_elementwise_vs_oracle():
    """Every parameter gradient of the full MatchaTTS train-step loss (dur + prior + diff, 32-true), element
    by element, against the CPU oracle restatement on the same recipe weights, batch and CFM randomness
    (the fixtures pin gradient norms; this pins the entries)."""
    import oracle_bind as OB
    from matcha.models.matcha_tts import MatchaTTS
    from matcha.training import synthetic_batch
    from oracle import matcha_oracle as MO

    def mp(value, mask):
        return torch.from_numpy(OB.maximum_path(value.detach().float().numpy(), mask.detach().float().numpy())[0])

    B, Tx, Ty = 4, 24, 96
    b = synthetic_batch(B, Tx, Ty, seed=91, device="cpu")
    gen = torch.Generator().manual_seed(92)
    t, z = torch.rand(B, 1, 1, generator=gen), torch.randn(B, 80, Ty, generator=gen)
    ref = MO.MatchaTTSOracle(150, 80, 192, maximum_path=mp)
    apply_recipe(ref, 93)
    ref.eval()
    out = ref(b["x"], b["x_lengths"], b["y"], b["y_lengths"], t=t, z=z)
    (out[0] + out[1] + out[2]).backward()
    want = {n: p.grad for n, p in ref.named_parameters() if p.grad is not None}

    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
    apply_recipe(model, 93)
    model.eval()
    d = lambda v: v.to(DEV)  # noqa: E731
    got_out = model(d(b["x"]), d(b["x_lengths"]), d(b["y"]), d(b["y_lengths"]), t=d(t), z=d(z))
    np.testing.assert_array_equal(got_out[3].cpu().numpy(), out[3].numpy())  # the same alignment
    (got_out[0] + got_out[1] + got_out[2]).backward()
    got = {n: p.grad.cpu() for n, p in model.named_parameters() if p.grad is not None}
    assert set(got) == set(want)
    worst = 0.0
    for n, g in want.items():
        scale = g.abs().max().item()
        err = (got[n] - g).abs().max().item()
        worst = max(worst, err / max(scale, 1e-30))
        assert err <= 2e-4 * scale + 1e-8, (n, err, scale)
    print(f"worst element-wise gradient error / tensor max: {worst:.2e} over {len(want)} tensors")


def test_decoder_more_than_eight_resnets_vs_oracle():
    """channels=(32, 32, 32), num_mid_blocks=3: nine Resnet1D blocks, so the time path's stacked
    projections run as two rows-linear launches (8 + 1 matrices) forward and backward."""
    from matcha.models.components.decoder import Decoder
    from oracle.matcha_oracle import DecoderOracle

    kw = dict(channels=(32, 32, 32), attention_head_dim=16, num_heads=2, num_mid_blocks=3)
    dec = Decoder(16, 8, **kw).to(DEV)
    assert len(dec._resnets()) == 9
    ref = DecoderOracle(16, 8, **kw)
    apply_recipe(dec, 5)
    apply_recipe(ref, 5)
    dec.eval()
    ref.eval()
    g = torch.Generator().manual_seed(9)
    B, T = 2, 48
    x, mu = torch.randn(B, 8, T, generator=g), torch.randn(B, 8, T, generator=g)
    mask = (torch.arange(T)[None, None] < torch.tensor([48, 37])[:, None, None]).float()
    t = torch.rand(B, generator=g)
    xd, mud = x.to(DEV).requires_grad_(True), mu.to(DEV)
    u = dec(xd, mask.to(DEV), mud, t.to(DEV))
    (u.square().sum()).backward()
    xr = x.clone().requires_grad_(True)
    ur = ref(xr, mask, mu, t)
    (ur.square().sum()).backward()
    assert rel(u.detach().cpu().numpy(), ur.detach().numpy()) < 1e-4
    assert rel(xd.grad.cpu().numpy(), xr.grad.numpy()) < 1e-3
    got = dict(dec.named_parameters())
    for name, p in ref.named_parameters():
        if "mlp" in name or "time_mlp" in name:  # the chunked time path's weight / bias gradients
            assert rel(got[name].grad.cpu().numpy(), p.grad.numpy()) < 1e-3, name
