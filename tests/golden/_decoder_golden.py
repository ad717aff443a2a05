"""Decoder / CFM / MatchaTTS golden fixtures, produced by running the REFERENCE model code
(/root/reference/matcha/...) on CPU in fp32, eval mode (dropout off), with injected RNG.

The reference imports diffusers 0.25 (transformer.py:13-23, not vendored, not installed here) and
pytorch_lightning (baselightningmodule.py:10-11, not installed).  This script writes a small
restatement of exactly the symbols the reference uses into a temporary directory:
  diffusers.models.attention_processor.Attention  -- to_q/k/v Linear(bias=False), to_out=[Linear, Dropout],
      prepare_attention_mask = repeat_interleave(heads, dim=0) -> view(B, heads, -1, T), then
      F.scaled_dot_product_attention(q, k, v, attn_mask=<float mask>, dropout_p=0) (AttnProcessor2_0):
      a float 0/1 mask is an ADDITIVE bias (+1 on valid keys)
  diffusers.models.attention.GELU(dim_in, dim_out, approximate="none") = Linear + F.gelu
  GEGLU / ApproximateGELU / AdaLayerNorm* (imported, unused by the decoder), LoRACompatibleLinear,
  maybe_allow_in_graph
  pytorch_lightning.LightningModule = nn.Module with no-op save_hyperparameters/log/log_dict
Fidelity at the diffusers boundary therefore rests on this restatement ("parity unpinned" there, as
SURVEY 8c records); everything else is the reference's own code.
"""
from __future__ import annotations

import sys
import tempfile
import textwrap
from pathlib import Path
from types import SimpleNamespace

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
REF = Path("/root/reference")

SHIM = {
    "diffusers/__init__.py": "",
    "diffusers/models/__init__.py": "",
    "diffusers/utils/__init__.py": "",
    "diffusers/utils/torch_utils.py": "def maybe_allow_in_graph(cls):\n    return cls\n",
    "diffusers/models/lora.py": textwrap.dedent("""
        import torch.nn as nn
        class LoRACompatibleLinear(nn.Linear):
            def forward(self, hidden_states, scale: float = 1.0):
                return super().forward(hidden_states)
    """),
    "diffusers/models/attention.py": textwrap.dedent("""
        import torch
        import torch.nn as nn
        import torch.nn.functional as F
        class GELU(nn.Module):
            def __init__(self, dim_in, dim_out, approximate="none", bias=True):
                super().__init__()
                self.proj = nn.Linear(dim_in, dim_out, bias=bias)
                self.approximate = approximate
            def forward(self, hidden_states):
                return F.gelu(self.proj(hidden_states), approximate=self.approximate)
        class GEGLU(nn.Module):
            def __init__(self, dim_in, dim_out, bias=True):
                super().__init__()
                self.proj = nn.Linear(dim_in, dim_out * 2, bias=bias)
            def forward(self, hidden_states):
                h, gate = self.proj(hidden_states).chunk(2, dim=-1)
                return h * F.gelu(gate)
        class ApproximateGELU(nn.Module):
            def __init__(self, dim_in, dim_out, bias=True):
                super().__init__()
                self.proj = nn.Linear(dim_in, dim_out, bias=bias)
            def forward(self, x):
                x = self.proj(x)
                return x * torch.sigmoid(1.702 * x)
        class AdaLayerNorm(nn.Module):
            def __init__(self, *a, **k):
                raise NotImplementedError("unused by the Matcha decoder")
        class AdaLayerNormZero(AdaLayerNorm):
            pass
    """),
    "diffusers/models/attention_processor.py": textwrap.dedent("""
        import torch.nn as nn
        import torch.nn.functional as F
        class Attention(nn.Module):
            def __init__(self, query_dim, cross_attention_dim=None, heads=8, dim_head=64, dropout=0.0,
                         bias=False, upcast_attention=False, upcast_softmax=False, out_bias=True, **kw):
                super().__init__()
                inner = dim_head * heads
                kv_dim = cross_attention_dim if cross_attention_dim is not None else query_dim
                self.heads = heads
                self.to_q = nn.Linear(query_dim, inner, bias=bias)
                self.to_k = nn.Linear(kv_dim, inner, bias=bias)
                self.to_v = nn.Linear(kv_dim, inner, bias=bias)
                self.to_out = nn.ModuleList([nn.Linear(inner, query_dim, bias=out_bias), nn.Dropout(dropout)])
            def prepare_attention_mask(self, attention_mask, target_length, batch_size, out_dim=3):
                if attention_mask is None:
                    return attention_mask
                if attention_mask.shape[-1] != target_length:
                    attention_mask = F.pad(attention_mask, (0, target_length), value=0.0)
                if attention_mask.shape[0] < batch_size * self.heads:
                    attention_mask = attention_mask.repeat_interleave(self.heads, dim=0)
                return attention_mask
            def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None, **kw):
                b, s, _ = hidden_states.shape if encoder_hidden_states is None else encoder_hidden_states.shape
                if attention_mask is not None:
                    attention_mask = self.prepare_attention_mask(attention_mask, s, b)
                    attention_mask = attention_mask.view(b, self.heads, -1, attention_mask.shape[-1])
                q = self.to_q(hidden_states)
                ctx = hidden_states if encoder_hidden_states is None else encoder_hidden_states
                k = self.to_k(ctx)
                v = self.to_v(ctx)
                hd = k.shape[-1] // self.heads
                q = q.view(b, -1, self.heads, hd).transpose(1, 2)
                k = k.view(b, -1, self.heads, hd).transpose(1, 2)
                v = v.view(b, -1, self.heads, hd).transpose(1, 2)
                o = F.scaled_dot_product_attention(q, k, v, attn_mask=attention_mask, dropout_p=0.0, is_causal=False)
                o = o.transpose(1, 2).reshape(b, -1, self.heads * hd).to(q.dtype)
                o = self.to_out[0](o)
                return self.to_out[1](o)
    """),
    "pytorch_lightning/__init__.py": textwrap.dedent("""
        import torch.nn as nn
        class LightningModule(nn.Module):
            def save_hyperparameters(self, *a, **k):
                pass
            def log(self, *a, **k):
                pass
            def log_dict(self, *a, **k):
                pass
    """),
    "pytorch_lightning/utilities/__init__.py": "def grad_norm(module, norm_type=2):\n    return {}\n",
}


def install_shims() -> Path:
    d = Path(tempfile.mkdtemp(prefix="mtts_ref_shim_"))
    for rel, src in SHIM.items():
        p = d / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(src)
    sys.path.insert(0, str(REF))
    sys.path.insert(0, str(d))
    # the compiled reference Cython as matcha.utils.monotonic_align.core (else the reference silently
    # falls back to its pure-Python DP with the opposite tie rule, __init__.py:4-8)
    from make_golden import load_cython_core

    sys.modules["matcha.utils.monotonic_align.core"] = load_cython_core()
    return d


def ragged_mask(B, T, lengths):
    import torch

    m = torch.zeros(B, 1, T)
    for b, L in enumerate(lengths):
        m[b, :, :L] = 1.0
    return m


def decoder_case(out, prefix, dec_params, n_feats, B, T, lengths, seed, full_grads):
    import torch

    from matcha.models.components.flow_matching import ConditionalFlowMatching
    from weights_recipe import apply_recipe

    cfm = ConditionalFlowMatching(in_channels=2 * n_feats, out_channel=n_feats,
                                  cfm_params=SimpleNamespace(solver="euler", sigma_min=1e-4),
                                  decoder_params=dec_params)
    apply_recipe(cfm, seed)
    cfm.eval()
    g = torch.Generator().manual_seed(seed + 1)
    mask = ragged_mask(B, T, lengths)
    x1 = torch.randn(B, n_feats, T, generator=g) * mask
    mu = torch.randn(B, n_feats, T, generator=g)
    phi = torch.randn(B, n_feats, T, generator=g)
    tt = torch.rand(B, generator=g)
    with torch.no_grad():
        u = cfm.estimator(phi, mask, mu, tt)
    # compute_loss draws t then z (flow_matching.py:130,133): record them by replaying the seed
    torch.manual_seed(seed + 2)
    t_inj = torch.rand([B, 1, 1])
    z_inj = torch.randn_like(x1)
    torch.manual_seed(seed + 2)
    mu_r = mu.clone().requires_grad_(True)
    loss, phi_t = cfm.compute_loss(x1=x1, mask=mask, mu=mu_r)
    loss.backward()
    out[prefix + "mask"] = mask.numpy()
    out[prefix + "x1"], out[prefix + "mu"], out[prefix + "phi"] = x1.numpy(), mu.numpy(), phi.numpy()
    out[prefix + "t"] = tt.numpy()
    out[prefix + "u"] = u.numpy()
    out[prefix + "loss_t"], out[prefix + "loss_z"] = t_inj.numpy(), z_inj.numpy()
    out[prefix + "loss"] = np.array(loss.item(), np.float64)
    out[prefix + "phi_t"] = phi_t.detach().numpy()
    out[prefix + "grad_mu"] = mu_r.grad.numpy()
    names = [n for n, _ in cfm.named_parameters()]
    out[prefix + "param_names"] = np.array(names)
    out[prefix + "grad_norms"] = np.array([p.grad.double().norm().item() for _, p in cfm.named_parameters()])
    if full_grads:
        for n, p in cfm.named_parameters():
            out[prefix + "grad." + n] = p.grad.numpy()


def model_case(out, seed=13):
    import torch

    from matcha.models.matcha_tts import MatchaTTS
    from weights_recipe import apply_recipe

    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192)
    apply_recipe(model, seed)
    model.eval()
    g = torch.Generator().manual_seed(seed + 1)
    B, Tx, Ty = 2, 12, 48
    x_lengths = torch.tensor([12, 9])
    y_lengths = torch.tensor([48, 37])
    x = torch.randint(1, 150, (B, Tx), generator=g)
    for b in range(B):
        x[b, x_lengths[b]:] = 0
    y = torch.randn(B, 80, Ty, generator=g)
    for b in range(B):
        y[b, :, y_lengths[b]:] = 0
    torch.manual_seed(seed + 2)
    t_inj = torch.rand([B, 1, 1])
    z_inj = torch.randn(B, 80, Ty)
    with torch.no_grad():
        mu_x, logw, x_mask = model.encoder(x, x_lengths)
    torch.manual_seed(seed + 2)
    dur, prior, diff, attn = model(x=x, x_lengths=x_lengths, y=y, y_lengths=y_lengths)
    (dur + prior + diff).backward()
    out["m_x"], out["m_x_lengths"], out["m_y"], out["m_y_lengths"] = x.numpy(), x_lengths.numpy(), y.numpy(), y_lengths.numpy()
    out["m_t"], out["m_z"] = t_inj.numpy(), z_inj.numpy()
    out["m_mu_x"], out["m_logw"], out["m_x_mask"] = mu_x.numpy(), logw.numpy(), x_mask.numpy()
    out["m_losses"] = np.array([dur.item(), prior.item(), diff.item()], np.float64)
    out["m_attn"] = attn.detach().numpy().astype(np.int8)
    out["m_param_names"] = np.array([n for n, _ in model.named_parameters()])
    out["m_grad_norms"] = np.array([p.grad.double().norm().item() if p.grad is not None else 0.0
                                    for _, p in model.named_parameters()])
    out["m_nparams"] = np.array([sum(p.numel() for p in model.encoder.parameters()),
                                 sum(p.numel() for p in model.decoder.parameters())], np.int64)


def headline_case(out, seed=41, B=4, Tx=120, Ty=600):
    """BASELINE config 3's shape (Tx=120, Ty=600) at B=4: the reference MatchaTTS.forward
    (matcha_tts.py:247-325) in fp32 eval mode with t / z replayed from the seed
    (flow_matching.py:130,133): losses, the MAS alignment and per-parameter gradient norms."""
    import torch

    from matcha.models.matcha_tts import MatchaTTS
    from weights_recipe import apply_recipe

    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192)
    apply_recipe(model, seed)
    model.eval()
    g = torch.Generator().manual_seed(seed + 1)
    # lengths U[0.7 max, max] with element 0 = max
    x_lengths = torch.tensor([Tx] + [int(v) for v in torch.randint(int(0.7 * Tx), Tx + 1, (B - 1,), generator=g)])
    y_lengths = torch.tensor([Ty] + [int(v) for v in torch.randint(int(0.7 * Ty), Ty + 1, (B - 1,), generator=g)])
    x = torch.randint(1, 150, (B, Tx), generator=g) * (torch.arange(Tx)[None] < x_lengths[:, None])
    y = torch.randn(B, 80, Ty, generator=g) * (torch.arange(Ty)[None, None] < y_lengths[:, None, None])
    torch.manual_seed(seed + 2)
    t_inj = torch.rand([B, 1, 1])
    z_inj = torch.randn(B, 80, Ty)
    torch.manual_seed(seed + 2)
    dur, prior, diff, attn = model(x=x, x_lengths=x_lengths, y=y, y_lengths=y_lengths)
    (dur + prior + diff).backward()
    out["h_x"], out["h_x_lengths"], out["h_y"], out["h_y_lengths"] = x.numpy(), x_lengths.numpy(), y.numpy(), y_lengths.numpy()
    out["h_t"], out["h_z"] = t_inj.numpy(), z_inj.numpy()
    out["h_losses"] = np.array([dur.item(), prior.item(), diff.item()], np.float64)
    out["h_attn_rows"] = attn_row_starts(attn.detach().numpy())
    out["h_param_names"] = np.array([n for n, _ in model.named_parameters()])
    out["h_grad_norms"] = np.array([p.grad.double().norm().item() if p.grad is not None else 0.0
                                    for _, p in model.named_parameters()])


def attn_row_starts(attn):
    """[B, Tx, Ty] 0/1 monotone path -> int32 [B, Tx] first column of each row (-1: empty row)."""
    B, Tx, _ = attn.shape
    rows = np.full((B, Tx), -1, np.int32)
    for b in range(B):
        for x in range(Tx):
            nz = np.flatnonzero(attn[b, x])
            if nz.size:
                rows[b, x] = nz[0]
                assert np.all(attn[b, x, nz[0]:nz[-1] + 1] == 1)
    return rows


def synth_case(out, prefix, seed, B, Tx, x_lengths, n_timesteps, length_scale, temperature=1.0):
    """The reference MatchaTTS.synthesise (matcha_tts.py:178-245: encoder, ceil'd durations,
    generate_path, Euler ODE flow_matching.py:42-104) run from a seed; the Gaussian draw
    z = randn_like(mu) * temperature (flow_matching.py:60) is replayed from the same seed."""
    import torch

    from matcha.models.matcha_tts import MatchaTTS
    from weights_recipe import apply_recipe

    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192)
    apply_recipe(model, seed)
    model.eval()
    g = torch.Generator().manual_seed(seed + 1)
    xl = torch.tensor(x_lengths)
    x = torch.randint(1, 150, (B, Tx), generator=g) * (torch.arange(Tx)[None] < xl[:, None])
    # record the reference's own draw: z = randn_like(mu) (flow_matching.py:60), then * temperature
    drawn = []
    real_randn_like = torch.randn_like

    def recording_randn_like(*a, **k):
        drawn.append(real_randn_like(*a, **k))
        return drawn[-1]

    torch.manual_seed(seed + 2)
    torch.randn_like = recording_randn_like
    try:
        res = model.synthesise(x, xl, n_timesteps, temperature=temperature, length_scale=length_scale)
    finally:
        torch.randn_like = real_randn_like
    assert len(drawn) == 1
    z = drawn[0] * temperature
    out[prefix + "x"], out[prefix + "x_lengths"] = x.numpy(), xl.numpy()
    out[prefix + "z"] = z.numpy()
    out[prefix + "cfg"] = np.array([n_timesteps, length_scale, temperature], np.float64)
    for k in ("encoder_outputs", "decoder_outputs", "mel", "mel_lengths"):
        out[prefix + k] = res[k].numpy()
    out[prefix + "attn"] = res["attn"].numpy().astype(np.int8)


def main_headline():
    install_shims()
    sys.path.insert(0, str(HERE))
    import torch

    torch.set_num_threads(8)
    out: dict[str, np.ndarray] = {}
    headline_case(out)
    np.savez_compressed(HERE / "headline_golden.npz", **out)
    print("wrote headline_golden.npz", out["h_losses"])


def main_synth():
    install_shims()
    sys.path.insert(0, str(HERE))
    import torch

    torch.set_num_threads(8)
    out: dict[str, np.ndarray] = {}
    synth_case(out, "a_", 23, 2, 11, [11, 8], 4, 1.0)
    synth_case(out, "b_", 29, 3, 17, [17, 12, 5], 6, 2.0, temperature=0.667)
    np.savez_compressed(HERE / "synth_golden.npz", **out)
    print("wrote synth_golden.npz", {k: v.shape for k, v in out.items()})


def main():
    install_shims()
    sys.path.insert(0, str(HERE))
    import torch

    torch.set_num_threads(8)
    small = dict(channels=(32, 32), dropout=0.05, attention_head_dim=16, n_blocks=1, num_mid_blocks=2,
                 num_heads=2)
    full = dict(channels=(256, 256), dropout=0.05, attention_head_dim=64, n_blocks=1, num_mid_blocks=2,
                num_heads=4)
    out: dict[str, np.ndarray] = {}
    decoder_case(out, "s64_", small, 8, 2, 64, [64, 51], 11, True)
    decoder_case(out, "s65_", small, 8, 2, 65, [65, 40], 21, True)
    decoder_case(out, "s33_", small, 8, 3, 33, [33, 20, 7], 31, True)
    decoder_case(out, "f97_", full, 80, 2, 97, [97, 70], 12, False)
    np.savez_compressed(HERE / "decoder_golden.npz", **out)
    print("wrote decoder_golden.npz")
    out = {}
    model_case(out)
    np.savez_compressed(HERE / "model_golden.npz", **out)
    print("wrote model_golden.npz", out["m_losses"], out["m_nparams"])
