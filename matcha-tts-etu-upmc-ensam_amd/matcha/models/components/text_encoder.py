"""Text encoder with duration predictor (drop-in for matcha/models/components/text_encoder.py).

Reference: ConvReluNorm :17-57, DurationPredictor :60-96, RotaryPositionalEmbeddings :99-143,
MultiHeadAttention :146-230, FFN :235-253, Encoder :256-322, TextEncoder :325-402.  Same module tree
and parameter names.  Not a kernel target in this tier: it runs as PyTorch-ROCm
device ops, with the q/k/v 1x1 convs fused into one GEMM and scaled-dot-product attention (the
reference's masked_fill(-1e4) becomes an additive -1e4 bias; identical on valid query rows, where
both underflow to exactly 0, and padded rows are zeroed by the following x*mask).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from matcha.utils.model import sequence_mask


def _ln_c(x, ln: nn.LayerNorm):  # LayerNorm over channels of a [B, C, T] tensor
    return F.layer_norm(x.transpose(1, 2), ln.normalized_shape, ln.weight, ln.bias, ln.eps).transpose(1, 2)


class ConvReluNorm(nn.Module):
    def __init__(self, input_channels, hidden_channels, output_channels, kernel_size, num_layers, dropout_rate):
        super().__init__()
        pad = kernel_size // 2
        self.convolutions = nn.ModuleList(
            [nn.Conv1d(input_channels if i == 0 else hidden_channels, hidden_channels, kernel_size, padding=pad)
             for i in range(num_layers)])
        self.normalizations = nn.ModuleList([nn.LayerNorm(hidden_channels) for _ in range(num_layers)])
        self.activation_dropout = nn.Sequential(nn.ReLU(), nn.Dropout(dropout_rate))
        self.projection = nn.Conv1d(hidden_channels, output_channels, 1)
        self.projection.weight.data.zero_()
        self.projection.bias.data.zero_()

    def forward(self, x, x_mask):
        res = x
        for conv, ln in zip(self.convolutions, self.normalizations):
            x = self.activation_dropout(_ln_c(conv(x * x_mask), ln))
        return (res + self.projection(x)) * x_mask


class DurationPredictor(nn.Module):
    def __init__(self, input_channels, filter_channels, kernel_size, dropout_rate):
        super().__init__()
        pad = kernel_size // 2
        self.dropout = nn.Dropout(dropout_rate)
        self.conv_layer_1 = nn.Conv1d(input_channels, filter_channels, kernel_size, padding=pad)
        self.norm_layer_1 = nn.LayerNorm(filter_channels)
        self.conv_layer_2 = nn.Conv1d(filter_channels, filter_channels, kernel_size, padding=pad)
        self.norm_layer_2 = nn.LayerNorm(filter_channels)
        self.output_projection = nn.Conv1d(filter_channels, 1, 1)

    def forward(self, x, x_mask):
        x = self.dropout(_ln_c(torch.relu(self.conv_layer_1(x * x_mask)), self.norm_layer_1))
        x = self.dropout(_ln_c(torch.relu(self.conv_layer_2(x * x_mask)), self.norm_layer_2))
        return self.output_projection(x * x_mask) * x_mask


class RotaryPositionalEmbeddings(nn.Module):
    """Rotates the first ``feature_dim`` features of [B, H, T, d] (neg-half form, base 1e4)."""

    def __init__(self, feature_dim, base_freq=10_000):
        super().__init__()
        self.base_freq = base_freq
        self.feature_dim = int(feature_dim)
        self._cache = None

    def _tables(self, T, device):
        c = self._cache
        if c is None or c[0].shape[0] < T or c[0].device != device:
            theta = 1.0 / (self.base_freq ** (torch.arange(0, self.feature_dim, 2, device=device).float()
                                              / self.feature_dim))
            ang = torch.arange(T, device=device).float()[:, None] * theta[None, :]
            ang = torch.cat([ang, ang], dim=1)
            self._cache = c = (ang.cos(), ang.sin())
        return c[0][:T], c[1][:T]

    def forward(self, x):
        d = self.feature_dim
        cos, sin = self._tables(x.shape[2], x.device)
        xr, xp = x[..., :d], x[..., d:]
        h = d // 2
        neg = torch.cat([-xr[..., h:], xr[..., :h]], dim=-1)
        return torch.cat([xr * cos + neg * sin, xp], dim=-1)


class MultiHeadAttention(nn.Module):
    def __init__(self, channels, output_channels, num_heads, heads_share=True, dropout_rate=0.0,
                 proximal_bias=False, proximal_init=False):
        super().__init__()
        assert channels % num_heads == 0
        if proximal_bias:
            raise NotImplementedError("proximal_bias is not used by the Matcha encoder")
        self.num_heads = num_heads
        self.head_dim = channels // num_heads
        self.dropout_rate = dropout_rate
        self.query_conv = nn.Conv1d(channels, channels, 1)
        self.key_conv = nn.Conv1d(channels, channels, 1)
        self.value_conv = nn.Conv1d(channels, channels, 1)
        self.query_rope = RotaryPositionalEmbeddings(self.head_dim * 0.5)
        self.key_rope = RotaryPositionalEmbeddings(self.head_dim * 0.5)
        self.output_conv = nn.Conv1d(channels, output_channels, 1)
        nn.init.xavier_uniform_(self.query_conv.weight)
        nn.init.xavier_uniform_(self.key_conv.weight)
        if proximal_init:
            self.key_conv.weight.data.copy_(self.query_conv.weight.data)
            self.key_conv.bias.data.copy_(self.query_conv.bias.data)
        nn.init.xavier_uniform_(self.value_conv.weight)

    def forward(self, x, context, attention_bias):
        """x [B, C, T]; attention_bias [B, 1, T, T] additive (0 valid, -1e4 masked)."""
        B, C, T = x.shape
        H, d = self.num_heads, self.head_dim
        w = torch.cat([self.query_conv.weight, self.key_conv.weight, self.value_conv.weight], 0)[..., 0]
        b = torch.cat([self.query_conv.bias, self.key_conv.bias, self.value_conv.bias], 0)
        qkv = F.linear(x.transpose(1, 2), w, b)  # [B, T, 3C]
        q, k, v = (t.view(B, T, H, d).transpose(1, 2) for t in qkv.split(C, dim=-1))
        q, k = self.query_rope(q), self.key_rope(k)
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=attention_bias,
                                           dropout_p=self.dropout_rate if self.training else 0.0)
        o = o.transpose(1, 2).reshape(B, T, C)
        return F.linear(o, self.output_conv.weight[..., 0], self.output_conv.bias).transpose(1, 2)


class FFN(nn.Module):
    def __init__(self, input_channels, output_channels, filter_channels, kernel_size, dropout_rate=0.0):
        super().__init__()
        pad = kernel_size // 2
        self.conv_net = nn.Sequential(
            nn.Conv1d(input_channels, filter_channels, kernel_size, padding=pad), nn.ReLU(), nn.Dropout(dropout_rate),
            nn.Conv1d(filter_channels, output_channels, kernel_size, padding=pad), nn.Dropout(dropout_rate))

    def forward(self, x, x_mask):
        return self.conv_net(x * x_mask) * x_mask


class Encoder(nn.Module):
    def __init__(self, hidden_channels, filter_channels, num_heads, num_layers, kernel_size=1, dropout_rate=0.0,
                 **kwargs):
        super().__init__()
        self.num_layers = num_layers
        self.dropout = nn.Dropout(dropout_rate)
        self.attention_layers = nn.ModuleList(
            [MultiHeadAttention(hidden_channels, hidden_channels, num_heads, dropout_rate=dropout_rate)
             for _ in range(num_layers)])
        self.norm_layers_1 = nn.ModuleList([nn.LayerNorm(hidden_channels) for _ in range(num_layers)])
        self.ffn_layers = nn.ModuleList(
            [FFN(hidden_channels, hidden_channels, filter_channels, kernel_size, dropout_rate=dropout_rate)
             for _ in range(num_layers)])
        self.norm_layers_2 = nn.ModuleList([nn.LayerNorm(hidden_channels) for _ in range(num_layers)])

    def forward(self, x, x_mask):
        m2 = x_mask.unsqueeze(2) * x_mask.unsqueeze(-1)  # [B, 1, T, T]
        bias = torch.zeros_like(m2).masked_fill(m2 == 0, -1e4)
        for i in range(self.num_layers):
            x = x * x_mask
            a = self.dropout(self.attention_layers[i](x, x, bias))
            x = _ln_c(x + a, self.norm_layers_1[i])
            f = self.dropout(self.ffn_layers[i](x, x_mask))
            x = _ln_c(x + f, self.norm_layers_2[i])
        return x * x_mask


class TextEncoder(nn.Module):
    def __init__(self, encoder_type, encoder_params, duration_predictor_params, n_vocab):
        super().__init__()
        self.encoder_type = encoder_type
        self.vocab_size = n_vocab
        self.feature_dim = encoder_params.n_feats
        self.channel_dim = encoder_params.n_channels
        self.embedding = nn.Embedding(n_vocab, self.channel_dim)
        nn.init.normal_(self.embedding.weight, 0.0, self.channel_dim ** -0.5)
        if encoder_params.prenet:
            self.prenet = ConvReluNorm(self.channel_dim, self.channel_dim, self.channel_dim, kernel_size=5,
                                       num_layers=3, dropout_rate=0.1)
        else:
            self.prenet = lambda x, x_mask: x
        self.encoder = Encoder(self.channel_dim, encoder_params.filter_channels, encoder_params.n_heads,
                               encoder_params.n_layers, encoder_params.kernel_size, encoder_params.p_dropout)
        self.mean_projection = nn.Conv1d(self.channel_dim, self.feature_dim, 1)
        self.duration_predictor = DurationPredictor(self.channel_dim, duration_predictor_params.filter_channels_dp,
                                                    duration_predictor_params.kernel_size,
                                                    duration_predictor_params.p_dropout)

    def forward(self, text_input, text_lengths):
        emb = (self.embedding(text_input) * math.sqrt(self.channel_dim)).transpose(1, -1)
        mask = sequence_mask(text_lengths, emb.size(2)).unsqueeze(1).to(emb.dtype)
        h = self.encoder(self.prenet(emb, mask), mask)
        mu = self.mean_projection(h) * mask
        logw = self.duration_predictor(h.detach(), mask)
        return mu, logw, mask
