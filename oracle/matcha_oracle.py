"""oracle/matcha_oracle.py -- TEST INFRASTRUCTURE ONLY (the checker, never the product).

Plain fp32 PyTorch restatement (channel-major, exactly the reference's op order) of the Matcha-TTS
training forward:
  decoder        /root/reference/matcha/models/components/decoder.py:8-371
  transformer    /root/reference/matcha/models/components/transformer.py:105-370 (+ diffusers 0.25
                 Attention/AttnProcessor2_0 and GELU, restated: SDPA with a float 0/1 mask is an
                 additive bias, erf GELU)
  CFM loss       /root/reference/matcha/models/components/flow_matching.py:106-151
  text encoder   /root/reference/matcha/models/components/text_encoder.py:17-402
  model forward  /root/reference/matcha/models/matcha_tts.py:247-325 (simple-params init :294-366)
  utilities      /root/reference/matcha/utils/model.py:13-135
Parameter names equal the reference's, so a state_dict moves between reference, oracle and product.
Dropout layers sit where the reference has them (decoder 0.05, encoder 0.1) and are active only in
train mode: parity tests run eval(); bench.py's cpu_baseline times the train-mode step.
MAS inside MatchaTTSOracle.forward is the C oracle (oracle/mas_oracle.c) via tests/oracle_bind.py.

Pinned by tests/test_oracle_golden.py / tests/test_model_oracle.py against decoder_golden.npz and
model_golden.npz, which tests/golden/make_golden.py produced by running the reference code itself.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------------------- decoder pieces
def sinusoidal_embedding(t: torch.Tensor, dim: int, scale: float = 1000.0) -> torch.Tensor:
    """decoder.py:22-31"""
    if t.ndim < 1:
        t = t.unsqueeze(0)
    half = dim // 2
    freq = torch.exp(torch.arange(half, dtype=torch.float32) * -(math.log(10000.0) / (half - 1)))
    arg = scale * t.unsqueeze(1) * freq.unsqueeze(0)
    return torch.cat([arg.sin(), arg.cos()], dim=-1)


class TimeMLP(nn.Module):  # decoder.py:33-49
    def __init__(self, cin, cout):
        super().__init__()
        self.linear_1 = nn.Linear(cin, cout)
        self.linear_2 = nn.Linear(cout, cout)

    def forward(self, s):
        return self.linear_2(F.silu(self.linear_1(s)))


class ConvGNMish(nn.Module):  # Block1D, decoder.py:51-66
    def __init__(self, cin, cout):
        super().__init__()
        self.block = nn.Sequential(nn.Conv1d(cin, cout, 3, padding=1), nn.GroupNorm(8, cout), nn.Mish())

    def forward(self, x, m):
        return self.block(x * m) * m


class ResBlock(nn.Module):  # Resnet1D, decoder.py:68-86
    def __init__(self, cin, cout, tdim):
        super().__init__()
        self.mlp = nn.Sequential(nn.Mish(), nn.Linear(tdim, cout))
        self.block1 = ConvGNMish(cin, cout)
        self.block2 = ConvGNMish(cout, cout)
        self.res_conv = nn.Conv1d(cin, cout, 1)

    def forward(self, x, m, temb):
        h = self.block1(x, m) + self.mlp(temb)[:, :, None]
        return self.block2(h, m) + self.res_conv(x * m)  # not re-masked (:85)


class Down(nn.Module):  # Downsample1D, decoder.py:88-98
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv1d(c, c, 3, stride=2, padding=1)

    def forward(self, x):
        return self.conv(x)


class Up(nn.Module):  # Upsample1D, decoder.py:100-116
    def __init__(self, c):
        super().__init__()
        self.conv = nn.ConvTranspose1d(c, c, 4, 2, 1)

    def forward(self, x):
        return self.conv(x)


class Attn(nn.Module):
    """diffusers 0.25 Attention + AttnProcessor2_0 as used by transformer.py:251-259, 320-325."""

    def __init__(self, dim, heads, dim_head, dropout=0.0):
        super().__init__()
        inner = heads * dim_head
        self.heads = heads
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_k = nn.Linear(dim, inner, bias=False)
        self.to_v = nn.Linear(dim, inner, bias=False)
        self.to_out = nn.ModuleList([nn.Linear(inner, dim), nn.Dropout(dropout)])

    def forward(self, h, key_mask):
        B, T, _ = h.shape
        H = self.heads
        q = self.to_q(h).view(B, T, H, -1).transpose(1, 2)
        k = self.to_k(h).view(B, T, H, -1).transpose(1, 2)
        v = self.to_v(h).view(B, T, H, -1).transpose(1, 2)
        s = q @ k.transpose(-1, -2) / math.sqrt(q.shape[-1])
        s = s + key_mask[:, None, None, :]  # float 0/1 mask added, not masked
        o = torch.softmax(s, dim=-1) @ v
        return self.to_out[1](self.to_out[0](o.transpose(1, 2).reshape(B, T, -1)))


class GELUProj(nn.Module):  # diffusers GELU(dim, inner) : Linear + erf gelu
    def __init__(self, cin, cout):
        super().__init__()
        self.proj = nn.Linear(cin, cout)

    def forward(self, x):
        return F.gelu(self.proj(x))


class FF(nn.Module):  # FeedForward, transformer.py:105-188 (net = [GELU, Dropout, Linear])
    def __init__(self, dim, mult=4, dropout=0.0):
        super().__init__()
        self.net = nn.ModuleList([GELUProj(dim, dim * mult), nn.Dropout(dropout), nn.Linear(dim * mult, dim)])

    def forward(self, x):
        return self.net[2](self.net[1](self.net[0](x)))


class TBlock(nn.Module):  # BasicTransformerBlock (diffusers branch), transformer.py:297-370
    def __init__(self, dim, heads, dim_head, dropout=0.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim)
        self.attn1 = Attn(dim, heads, dim_head, dropout)
        self.norm3 = nn.LayerNorm(dim)
        self.ff = FF(dim, dropout=dropout)

    def forward(self, h, key_mask):
        h = self.attn1(self.norm1(h), key_mask) + h
        return self.ff(self.norm3(h)) + h


class DecoderOracle(nn.Module):
    """decoder.py:118-371 with the reference's module tree (hence its parameter names)."""

    def __init__(self, in_channels, out_channels, channels=(256, 256), dropout=0.05, attention_head_dim=64,
                 n_blocks=1, num_mid_blocks=2, num_heads=4):
        super().__init__()
        channels = tuple(channels)
        self.in_channels = in_channels
        tdim = channels[0] * 4
        self.time_mlp = TimeMLP(in_channels, tdim)

        def tblocks(c):
            return nn.ModuleList([TBlock(c, num_heads, attention_head_dim, dropout) for _ in range(n_blocks)])

        self.Downsampling_Blocks = nn.ModuleList()
        cout = in_channels
        for i, c in enumerate(channels):
            cin, cout = cout, c
            last = i == len(channels) - 1
            self.Downsampling_Blocks.append(nn.ModuleList([
                ResBlock(cin, cout, tdim), tblocks(cout),
                nn.Conv1d(cout, cout, 3, padding=1) if last else Down(cout)]))
        self.Mid_Blocks = nn.ModuleList(
            [nn.ModuleList([ResBlock(channels[-1], channels[-1], tdim), tblocks(channels[-1])])
             for _ in range(num_mid_blocks)])
        rev = channels[::-1] + (channels[0],)
        self.Upsampling_Blocks = nn.ModuleList()
        for i in range(len(rev) - 1):
            last = i == len(rev) - 2
            self.Upsampling_Blocks.append(nn.ModuleList([
                ResBlock(2 * rev[i], rev[i + 1], tdim), tblocks(rev[i + 1]),
                nn.Conv1d(rev[i + 1], rev[i + 1], 3, padding=1) if last else Up(rev[i + 1])]))
        self.final_conv = nn.Conv1d(channels[0], channels[0], 3, padding=1)
        self.final_norm = nn.GroupNorm(8, channels[0])
        self.final_proj = nn.Conv1d(channels[0], out_channels, 1)

    def _tf(self, blocks, x, m):
        h = x.transpose(1, 2)
        km = m[:, 0, :]
        for blk in blocks:
            h = blk(h, km)
        return h.transpose(1, 2)

    def forward(self, x, mask, mu, t, cond=None):
        temb = self.time_mlp(sinusoidal_embedding(t, self.in_channels))
        x = torch.cat([x, mu], dim=1)  # einops pack "b * t" (:288)
        skips, masks = [], [mask]
        for res, tfs, down in self.Downsampling_Blocks:
            m = masks[-1]
            x = self._tf(tfs, res(x, m, temb), m)
            skips.append(x)
            x = down(x * m)
            keep = (m.shape[-1] + 1) // 2 if isinstance(down, Down) else m.shape[-1]
            masks.append(m[:, :, :keep])  # prefix slice, not a stride-2 subsample (:311-316)
        masks = masks[:-1]
        m = masks[-1]
        for res, tfs in self.Mid_Blocks:
            x = self._tf(tfs, res(x, m, temb), m)
        for res, tfs, up in self.Upsampling_Blocks:
            m = masks.pop()
            skip = skips.pop()
            if x.shape[-1] != skip.shape[-1]:
                x = F.interpolate(x, size=skip.shape[-1], mode="nearest")  # odd T (:338-339)
            x = torch.cat([x, skip], dim=1)
            x = self._tf(tfs, res(x, m, temb), m)
            x = up(x * m)
            new = m.shape[-1] * 2 if isinstance(up, Up) else x.shape[-1]
            m = F.interpolate(m, size=new, mode="nearest") if new > m.shape[-1] else m[:, :, :new]
        x = F.mish(self.final_norm(self.final_conv(x * m)))
        return self.final_proj(x * m) * mask


class CFMOracle(nn.Module):
    """flow_matching.py:154-189 (+ BaseConditionalFlowMatching.compute_loss :106-151)."""

    def __init__(self, in_channels, out_channel, cfm_params=None, decoder_params=None, n_spks=1, spk_emb_dim=64):
        super().__init__()
        self.sigma_min = getattr(cfm_params, "sigma_min", 1e-4) if cfm_params is not None else 1e-4
        self.estimator = DecoderOracle(in_channels, out_channel, **(decoder_params or {}))

    @torch.no_grad()
    def forward(self, mu, mask, n_timesteps, temperature=1.0, spks=None, cond=None, z=None):
        """flow_matching.py:42-65 + solve_ode_euler :67-104 (same t / dt recurrence); z injectable."""
        if z is None:
            z = torch.randn_like(mu) * temperature
        t_span = torch.linspace(0, 1, n_timesteps + 1, device=mu.device)
        x, t, dt = z, t_span[0], t_span[1] - t_span[0]
        for step in range(1, len(t_span)):
            x = x + dt * self.estimator(x, mask, mu, t, cond)
            t = t + dt
            if step < len(t_span) - 1:
                dt = t_span[step + 1] - t
        return x

    def compute_loss(self, x1, mask, mu, spks=None, cond=None, t=None, z=None):
        B = mu.shape[0]
        if t is None:
            t = torch.rand([B, 1, 1], dtype=mu.dtype)
        if z is None:
            z = torch.randn_like(x1)
        s = self.sigma_min
        phi = (1 - (1 - s) * t) * z + t * x1
        u = x1 - (1 - s) * z  # target is NOT masked
        pred = self.estimator(phi, mask, mu, t.squeeze(), cond)
        loss = F.mse_loss(pred, u, reduction="sum") / (torch.sum(mask) * u.shape[1])
        return loss, phi


# ----------------------------------------------------------------------------- text encoder
def sequence_mask(lengths, max_len=None):  # model.py:13-34
    if max_len is None:
        max_len = int(lengths.max())
    return torch.arange(max_len, dtype=lengths.dtype, device=lengths.device)[None, :] < lengths[:, None]


class ConvReluNormO(nn.Module):  # text_encoder.py:17-57
    def __init__(self, c, k=5, n=3, p=0.1):
        super().__init__()
        self.drop = nn.Dropout(p)
        self.convolutions = nn.ModuleList([nn.Conv1d(c, c, k, padding=k // 2) for _ in range(n)])
        self.normalizations = nn.ModuleList([nn.LayerNorm(c) for _ in range(n)])
        self.projection = nn.Conv1d(c, c, 1)

    def forward(self, x, m):
        r = x
        for conv, ln in zip(self.convolutions, self.normalizations):
            x = self.drop(F.relu(ln(conv(x * m).transpose(1, 2)).transpose(1, 2)))
        return (r + self.projection(x)) * m


class DurationPredictorO(nn.Module):  # text_encoder.py:60-96
    def __init__(self, cin, cf, k, p=0.1):
        super().__init__()
        self.drop = nn.Dropout(p)
        self.conv_layer_1 = nn.Conv1d(cin, cf, k, padding=k // 2)
        self.norm_layer_1 = nn.LayerNorm(cf)
        self.conv_layer_2 = nn.Conv1d(cf, cf, k, padding=k // 2)
        self.norm_layer_2 = nn.LayerNorm(cf)
        self.output_projection = nn.Conv1d(cf, 1, 1)

    def forward(self, x, m):
        x = self.drop(self.norm_layer_1(torch.relu(self.conv_layer_1(x * m)).transpose(1, 2)).transpose(1, 2))
        x = self.drop(self.norm_layer_2(torch.relu(self.conv_layer_2(x * m)).transpose(1, 2)).transpose(1, 2))
        return self.output_projection(x * m) * m


def rope(x: torch.Tensor, rot_dim: int) -> torch.Tensor:
    """text_encoder.py:99-143 on [B,H,T,D]: rotate the first rot_dim features (neg-half form)."""
    T = x.shape[2]
    theta = 1.0 / (10000 ** (torch.arange(0, rot_dim, 2).float() / rot_dim))
    ang = torch.arange(T).float()[:, None] * theta[None, :]
    ang = torch.cat([ang, ang], dim=1)
    cos, sin = ang.cos(), ang.sin()
    xr, xp = x[..., :rot_dim], x[..., rot_dim:]
    half = rot_dim // 2
    neg = torch.cat([-xr[..., half:], xr[..., :half]], dim=-1)
    return torch.cat([xr * cos + neg * sin, xp], dim=-1)


class MHAO(nn.Module):  # text_encoder.py:146-230
    def __init__(self, c, heads, p=0.1):
        super().__init__()
        self.heads = heads
        self.drop = nn.Dropout(p)
        self.query_conv = nn.Conv1d(c, c, 1)
        self.key_conv = nn.Conv1d(c, c, 1)
        self.value_conv = nn.Conv1d(c, c, 1)
        self.output_conv = nn.Conv1d(c, c, 1)

    def forward(self, x, amask):
        B, C, T = x.shape
        H = self.heads
        d = C // H
        q = self.query_conv(x).view(B, H, d, T).transpose(2, 3)
        k = self.key_conv(x).view(B, H, d, T).transpose(2, 3)
        v = self.value_conv(x).view(B, H, d, T).transpose(2, 3)
        rd = int(d * 0.5)
        q, k = rope(q, rd), rope(k, rd)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(d)
        s = s.masked_fill(amask == 0, -1e4)
        o = self.drop(torch.softmax(s, dim=-1)) @ v
        return self.output_conv(o.transpose(2, 3).contiguous().view(B, C, T))


class FFNO(nn.Module):  # text_encoder.py:235-253
    def __init__(self, c, cf, k, p=0.1):
        super().__init__()
        self.conv_net = nn.Sequential(nn.Conv1d(c, cf, k, padding=k // 2), nn.ReLU(), nn.Dropout(p),
                                      nn.Conv1d(cf, c, k, padding=k // 2), nn.Dropout(p))

    def forward(self, x, m):
        return self.conv_net(x * m) * m


class EncoderO(nn.Module):  # text_encoder.py:256-322
    def __init__(self, c, cf, heads, layers, k):
        super().__init__()
        self.attention_layers = nn.ModuleList([MHAO(c, heads) for _ in range(layers)])
        self.norm_layers_1 = nn.ModuleList([nn.LayerNorm(c) for _ in range(layers)])
        self.ffn_layers = nn.ModuleList([FFNO(c, cf, k) for _ in range(layers)])
        self.norm_layers_2 = nn.ModuleList([nn.LayerNorm(c) for _ in range(layers)])
        self.drop = nn.Dropout(0.1)

    def forward(self, x, m):
        amask = m.unsqueeze(2) * m.unsqueeze(-1)
        for att, n1, ffn, n2 in zip(self.attention_layers, self.norm_layers_1, self.ffn_layers, self.norm_layers_2):
            x = x * m
            x = n1((x + self.drop(att(x, amask))).transpose(1, 2)).transpose(1, 2)
            x = n2((x + self.drop(ffn(x, m))).transpose(1, 2)).transpose(1, 2)
        return x * m


class TextEncoderO(nn.Module):  # text_encoder.py:325-402 (simple-params config, matcha_tts.py:104-176)
    def __init__(self, n_vocab, n_feats=80, c=192, cf=768, heads=2, layers=6, k=3, dp_filter=256):
        super().__init__()
        self.c = c
        self.embedding = nn.Embedding(n_vocab, c)
        self.prenet = ConvReluNormO(c)
        self.encoder = EncoderO(c, cf, heads, layers, k)
        self.mean_projection = nn.Conv1d(c, n_feats, 1)
        self.duration_predictor = DurationPredictorO(c, dp_filter, 3)

    def forward(self, x, x_lengths):
        e = (self.embedding(x) * math.sqrt(self.c)).transpose(1, -1)
        m = sequence_mask(x_lengths, e.size(2)).unsqueeze(1).to(e.dtype)
        h = self.encoder(self.prenet(e, m), m)
        return self.mean_projection(h) * m, self.duration_predictor(h.detach(), m), m


def generate_path(duration, mask):  # model.py:77-114 (build_alignment_path)
    B, Tx, Ty = mask.shape
    cum = torch.cumsum(duration, 1)
    path = sequence_mask(cum.reshape(B * Tx), Ty).to(mask.dtype).view(B, Tx, Ty)
    path = path - F.pad(path, (0, 0, 1, 0, 0, 0))[:, :-1]
    return path * mask


def fix_len_compatibility(length, num_downsamplings_in_unet=2):  # model.py:37-57
    f = 2 ** num_downsamplings_in_unet
    return int((torch.ceil(length / f) * f).item())


class MatchaTTSOracle(nn.Module):
    """MatchaTTS(n_vocab, out_channels=80, hidden_channels=192) forward (matcha_tts.py:247-325)."""

    def __init__(self, n_vocab=150, out_channels=80, hidden_channels=192, maximum_path=None):
        super().__init__()
        self.n_feats = out_channels
        self.encoder = TextEncoderO(n_vocab, out_channels, hidden_channels)
        self.decoder = CFMOracle(2 * out_channels, out_channels,
                                 decoder_params=dict(channels=(256, 256), attention_head_dim=64, num_heads=4))
        self.register_buffer("mel_mean", torch.tensor(0.0))
        self.register_buffer("mel_std", torch.tensor(1.0))
        self._maximum_path = maximum_path

    @torch.no_grad()
    def synthesise(self, x, x_lengths, n_timesteps, temperature=1.0, length_scale=1.0, z=None):
        """matcha_tts.py:179-245 (rtf omitted); ``z`` [B, n_feats, y_max_length_] injectable."""
        mu_x, logw, x_mask = self.encoder(x, x_lengths)
        w = torch.exp(logw) * x_mask
        w_ceil = torch.ceil(w) * length_scale
        y_lengths = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
        y_max_length = y_lengths.max()
        y_max_length_ = fix_len_compatibility(y_max_length)
        y_mask = sequence_mask(y_lengths, y_max_length_).unsqueeze(1).to(x_mask.dtype)
        attn_mask = x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)
        attn = generate_path(w_ceil.squeeze(1), attn_mask.squeeze(1)).unsqueeze(1)
        mu_y = torch.matmul(attn.squeeze(1).transpose(1, 2), mu_x.transpose(1, 2)).transpose(1, 2)
        out = self.decoder(mu_y, y_mask, n_timesteps, temperature, z=z)
        ym = int(y_max_length)
        return {"encoder_outputs": mu_y[:, :, :ym], "decoder_outputs": out[:, :, :ym], "attn": attn[:, :, :ym],
                "mel": out[:, :, :ym] * self.mel_std + self.mel_mean, "mel_lengths": y_lengths}

    def forward(self, x, x_lengths, y, y_lengths, out_size=None, cond=None, durations=None, t=None, z=None,
                return_log_prior=False):
        mu_x, logw, x_mask = self.encoder(x, x_lengths)
        y_mask = sequence_mask(y_lengths, y.shape[-1]).unsqueeze(1).to(x_mask)
        attn_mask = x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)
        with torch.no_grad():  # matcha_tts.py:276-285
            const = -0.5 * math.log(2 * math.pi) * self.n_feats
            factor = -0.5 * torch.ones(mu_x.shape, dtype=mu_x.dtype)
            y_square = torch.matmul(factor.transpose(1, 2), y ** 2)
            y_mu_double = torch.matmul(2.0 * (factor * mu_x).transpose(1, 2), y)
            mu_square = torch.sum(factor * (mu_x ** 2), 1).unsqueeze(-1)
            log_prior = y_square - y_mu_double + mu_square + const
            attn = self._maximum_path(log_prior, attn_mask.squeeze(1)).detach()
        logw_ = torch.log(1e-8 + torch.sum(attn.unsqueeze(1), -1)) * x_mask
        dur_loss = torch.sum((logw - logw_) ** 2) / torch.sum(x_lengths)
        mu_y = torch.matmul(attn.squeeze(1).transpose(1, 2), mu_x.transpose(1, 2)).transpose(1, 2)
        diff_loss, _ = self.decoder.compute_loss(x1=y, mask=y_mask, mu=mu_y, cond=cond, t=t, z=z)
        prior_loss = torch.sum(0.5 * ((y - mu_y) ** 2 + math.log(2 * math.pi)) * y_mask)
        prior_loss = prior_loss / (torch.sum(y_mask) * self.n_feats)
        if return_log_prior:
            return dur_loss, prior_loss, diff_loss, attn, log_prior
        return dur_loss, prior_loss, diff_loss, attn
