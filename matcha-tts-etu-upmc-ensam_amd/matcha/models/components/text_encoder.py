"""Text encoder with duration predictor (drop-in for matcha/models/components/text_encoder.py).

Reference: ConvReluNorm :17-57, DurationPredictor :60-96, RotaryPositionalEmbeddings :99-143,
MultiHeadAttention :146-230, FFN :235-253, Encoder :256-322, TextEncoder :325-402.  Same module tree
and parameter names (a reference checkpoint loads unchanged).

Runs token-major ([B, T, C]) on the same libmtts_hip kernels as the decoder:
  * every Conv1d is an implicit GEMM with the input mask as a row scale, ReLU / dropout / residual /
    output mask in the GEMM epilogue (k = 5 prenet convs included);
  * the prenet's LN -> ReLU -> Dropout and the duration predictor's LN -> Dropout are one LayerNorm
    kernel each way;
  * q/k/v are one GEMM over the stacked 1x1 conv weights, RoPE is one elementwise kernel on the fused
    projection, attention is the flash kernel (head dim 96) with dropout on the probabilities;
  * the FFN (conv k3 -> ReLU -> Dropout -> conv k3 -> Dropout, then the Encoder's Dropout and the
    residual) is two GEMMs (conv_ffn_tm).
Masking: the reference's masked_fill(mask == 0, -1e4) on the scores becomes an additive key bias
of -1e4 on padded keys.  On valid query rows the two are identical (both weights underflow to
exactly 0 in fp32); padded query rows differ, and padded rows are dead: every consumer masks them
(x * mask at each layer's input and at the end, the FFN and projections' masked inputs, -1e4 keys),
so no loss or gradient depends on them.  For the same reason residual adds use the unmasked input.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch
import torch.nn as nn

from matcha import _native as N
from matcha.models.components import _ops as O

# MTTS_ENCODER_DX_LINK=0: autograd sums each encoder layer's two input gradients (A/B switch)
_ENC_LINK = os.environ.get("MTTS_ENCODER_DX_LINK", "1") != "0"
# MTTS_QKV_BIAS_ONE_CAT=0: one q|k|v bias concatenation per layer (A/B switch)
_ONE_BIAS_CAT = os.environ.get("MTTS_QKV_BIAS_ONE_CAT", "1") != "0"


class ConvReluNorm(nn.Module):
    def __init__(self, input_channels, hidden_channels, output_channels, kernel_size, num_layers, dropout_rate):
        super().__init__()
        pad = kernel_size // 2
        self.dropout_rate = dropout_rate
        self.convolutions = nn.ModuleList(
            [nn.Conv1d(input_channels if i == 0 else hidden_channels, hidden_channels, kernel_size, padding=pad)
             for i in range(num_layers)])
        self.normalizations = nn.ModuleList([nn.LayerNorm(hidden_channels) for _ in range(num_layers)])
        self.activation_dropout = nn.Sequential(nn.ReLU(), nn.Dropout(dropout_rate))
        self.projection = nn.Conv1d(hidden_channels, output_channels, 1)
        self.projection.weight.data.zero_()
        self.projection.bias.data.zero_()

    def forward_tm(self, x, m):
        """x [B, T, C], m [B, T] -> (x + proj(h)) * m  (text_encoder.py:48-57)."""
        p = self.dropout_rate if self.training else 0.0
        h = x
        for conv, ln in zip(self.convolutions, self.normalizations):
            h = O.conv_tm(h, conv.weight, conv.bias, mask=m)
            h = O.layer_norm_tm(h, ln.weight, ln.bias, ln.eps, relu=True, dropout_p=p)
        return O.linear_tm(h, self.projection.weight, self.projection.bias, residual=x, out_scale=m)

    def forward(self, x, x_mask):
        return self.forward_tm(x.transpose(1, 2), x_mask[:, 0]).transpose(1, 2)


class DurationPredictor(nn.Module):
    def __init__(self, input_channels, filter_channels, kernel_size, dropout_rate):
        super().__init__()
        pad = kernel_size // 2
        self.dropout_rate = dropout_rate
        self.dropout = nn.Dropout(dropout_rate)
        self.conv_layer_1 = nn.Conv1d(input_channels, filter_channels, kernel_size, padding=pad)
        self.norm_layer_1 = nn.LayerNorm(filter_channels)
        self.conv_layer_2 = nn.Conv1d(filter_channels, filter_channels, kernel_size, padding=pad)
        self.norm_layer_2 = nn.LayerNorm(filter_channels)
        self.output_projection = nn.Conv1d(filter_channels, 1, 1)

    def forward_tm(self, x, m):
        """text_encoder.py:81-96: (conv -> ReLU -> LN -> Dropout) x 2 -> 1x1 conv, masked; -> [B, T, 1]."""
        p = self.dropout_rate if self.training else 0.0
        for conv, ln in ((self.conv_layer_1, self.norm_layer_1), (self.conv_layer_2, self.norm_layer_2)):
            x = O.conv_tm(x, conv.weight, conv.bias, mask=m, relu=True)
            x = O.layer_norm_tm(x, ln.weight, ln.bias, ln.eps, dropout_p=p)
        return O.linear_tm(x, self.output_projection.weight, self.output_projection.bias, in_scale=m, out_scale=m)

    def forward(self, x, x_mask):
        return self.forward_tm(x.transpose(1, 2), x_mask[:, 0]).transpose(1, 2)


class RotaryPositionalEmbeddings(nn.Module):
    """cos/sin tables of the reference's partial RoPE (text_encoder.py:99-143): the first feature_dim
    features of every head, rotate-half form, base 1e4.  The rotation itself is mtts_rope_qk."""

    def __init__(self, feature_dim, base_freq=10_000):
        super().__init__()
        self.base_freq = base_freq
        self.feature_dim = int(feature_dim)
        self._cache = None

    def tables(self, T: int, device) -> tuple[torch.Tensor, torch.Tensor]:
        """cos, sin [T, feature_dim / 2], the reference's fp32 formula (:109-126)."""
        c = self._cache
        if c is None or c[0].shape[0] < T or c[0].device != device:
            # fp32 even inside a bf16 autocast region (autocast would run the einsum in bf16)
            with torch.autocast(device_type=device.type, enabled=False):
                theta = 1.0 / (self.base_freq ** (torch.arange(0, self.feature_dim, 2).float()
                                                  / self.feature_dim)).to(device)
                ang = torch.einsum("n,d->nd", torch.arange(T, device=device).float(), theta)
                self._cache = c = (ang.cos().float().contiguous(), ang.sin().float().contiguous())
        return c[0][:T], c[1][:T]


class MultiHeadAttention(nn.Module):
    def __init__(self, channels, output_channels, num_heads, heads_share=True, dropout_rate=0.0,
                 proximal_bias=False, proximal_init=False):
        super().__init__()
        assert channels % num_heads == 0
        if proximal_bias:
            raise NotImplementedError("proximal_bias is not used by the Matcha encoder")
        self.channels = channels
        self.num_heads = num_heads
        self.head_dim = channels // num_heads
        self.dropout_rate = dropout_rate
        self.query_conv = nn.Conv1d(channels, channels, 1)
        self.key_conv = nn.Conv1d(channels, channels, 1)
        self.value_conv = nn.Conv1d(channels, channels, 1)
        self.query_rope = RotaryPositionalEmbeddings(self.head_dim * 0.5)
        self.key_rope = RotaryPositionalEmbeddings(self.head_dim * 0.5)
        self.output_conv = nn.Conv1d(channels, output_channels, 1)
        self.dropout = nn.Dropout(dropout_rate)
        nn.init.xavier_uniform_(self.query_conv.weight)
        nn.init.xavier_uniform_(self.key_conv.weight)
        if proximal_init:
            self.key_conv.weight.data.copy_(self.query_conv.weight.data)
            self.key_conv.bias.data.copy_(self.query_conv.bias.data)
        nn.init.xavier_uniform_(self.value_conv.weight)

    def qkv_bias(self):
        return torch.cat([self.query_conv.bias, self.key_conv.bias, self.value_conv.bias])

    def attend_tm(self, x, m, key_bias, qkv_bias=None, dx_link=None):
        """softmax-attention output [B, T, C] of (x * m) before output_conv (text_encoder.py:188-230).
        qkv_bias: the stacked q|k|v bias when the caller built every layer's at once.  dx_link: the
        projection's dgrad takes the linked gradient of x (O.GradLink)."""
        T = x.shape[1]
        qkv = O.linear_tm(x, (self.query_conv.weight, self.key_conv.weight, self.value_conv.weight),
                          self.qkv_bias() if qkv_bias is None else qkv_bias, in_scale=m, dx_link=dx_link,
                          dx_link_role="take" if dx_link is not None else None)
        cos, sin = self.query_rope.tables(T, x.device)  # query_rope and key_rope are the same rotation
        qkv = O.rope_tm(qkv, cos, sin, self.num_heads, self.query_rope.feature_dim)
        p = self.dropout_rate if self.training else 0.0
        return O.attention_tm(qkv, key_bias, self.num_heads, dropout_p=p)

    def forward(self, x, context, attention_mask=None):
        """Reference API: x [B, C, T] (context must be x: self-attention), attention_mask [B, 1, T, T]
        = x_mask_q * x_mask_k."""
        assert context is x, "the encoder uses self-attention only"
        m = attention_mask[:, 0].amax(dim=1) if attention_mask is not None else \
            torch.ones(x.shape[0], x.shape[2], device=x.device)
        o = self.attend_tm(x.transpose(1, 2), torch.ones_like(m), (m - 1.0) * 1e4)
        return O.linear_tm(o, self.output_conv.weight, self.output_conv.bias).transpose(1, 2)


class FFN(nn.Module):
    def __init__(self, input_channels, output_channels, filter_channels, kernel_size, dropout_rate=0.0):
        super().__init__()
        pad = kernel_size // 2
        self.dropout_rate = dropout_rate
        self.conv_net = nn.Sequential(
            nn.Conv1d(input_channels, filter_channels, kernel_size, padding=pad), nn.ReLU(), nn.Dropout(dropout_rate),
            nn.Conv1d(filter_channels, output_channels, kernel_size, padding=pad), nn.Dropout(dropout_rate))

    def forward_tm(self, x, m, residual=None, extra_dropout: float = 0.0):
        """(residual + Dropout_extra(FFN(x, m))) * m, token-major (text_encoder.py:247-253, 307-313)."""
        p = self.dropout_rate if self.training else 0.0
        keep_out = (1.0 - p) * (1.0 - extra_dropout)
        c1, c2 = self.conv_net[0], self.conv_net[3]
        return O.conv_ffn_tm(x, c1.weight, c1.bias, c2.weight, c2.bias, m, residual, p_in=p, p_out=1.0 - keep_out)

    def forward(self, x, x_mask):
        return self.forward_tm(x.transpose(1, 2), x_mask[:, 0]).transpose(1, 2)


class Encoder(nn.Module):
    def __init__(self, hidden_channels, filter_channels, num_heads, num_layers, kernel_size=1, dropout_rate=0.0,
                 **kwargs):
        super().__init__()
        self.num_layers = num_layers
        self.dropout_rate = dropout_rate
        self.dropout = nn.Dropout(dropout_rate)
        self.attention_layers = nn.ModuleList(
            [MultiHeadAttention(hidden_channels, hidden_channels, num_heads, dropout_rate=dropout_rate)
             for _ in range(num_layers)])
        self.norm_layers_1 = nn.ModuleList([nn.LayerNorm(hidden_channels) for _ in range(num_layers)])
        self.ffn_layers = nn.ModuleList(
            [FFN(hidden_channels, hidden_channels, filter_channels, kernel_size, dropout_rate=dropout_rate)
             for _ in range(num_layers)])
        self.norm_layers_2 = nn.ModuleList([nn.LayerNorm(hidden_channels) for _ in range(num_layers)])

    def forward_tm(self, h, m, key_bias=None):
        """text_encoder.py:296-322, token-major; returns the UNMASKED last LayerNorm output (callers
        apply the final x * mask through their input row scale).  key_bias: (m - 1) * 1e4 if the caller
        has it (O.sequence_mask_f32 makes both in one launch)."""
        p = self.dropout_rate if self.training else 0.0
        if key_bias is None:
            key_bias = (m - 1.0) * 1e4  # masked_fill(-1e4) on padded keys
        # every layer's stacked q|k|v bias from ONE concatenation (one launch instead of one per layer) --
        # except with the opt-in side-stream weight gradients: the concatenation routes the bias gradients
        # through autograd's SplitBackward, which reads them on the main stream while the side stream
        # still writes them; per layer each bias gradient is a direct view
        layers = list(self.attention_layers)
        if O._SIDE_WGRAD["on"] or not _ONE_BIAS_CAT:
            qkv_biases = [None] * len(layers)
        else:
            qkv_biases = torch.cat([b for a in layers for b in (a.query_conv.bias, a.key_conv.bias, a.value_conv.bias)])
            qkv_biases = qkv_biases.split([3 * a.query_conv.bias.numel() for a in layers])
        for attn, ln1, ffn, ln2, qb in zip(layers, self.norm_layers_1, self.ffn_layers, self.norm_layers_2, qkv_biases):
            # h feeds the masked q|k|v projection and output_conv's residual: the residual gradient is added in
            # the projection's dgrad epilogue ((acc + g) * m; g vanishes on masked rows: it is LN1's input
            # gradient, and LN1's output only reaches the loss through the FFN's masked output)
            link = O.GradLink() if _ENC_LINK and h.requires_grad and torch.is_grad_enabled() else None
            o = attn.attend_tm(h, m, key_bias, qkv_bias=qb, dx_link=link)
            x = O.linear_tm(o, attn.output_conv.weight, attn.output_conv.bias, residual=h, dropout_p=p,
                            dx_link=link, dx_link_role="give_res" if link is not None else None)
            x = O.layer_norm_tm(x, ln1.weight, ln1.bias, ln1.eps)
            x = ffn.forward_tm(x, m, residual=x, extra_dropout=p)
            h = O.layer_norm_tm(x, ln2.weight, ln2.bias, ln2.eps)
        return h

    def forward(self, x, x_mask):
        m = x_mask[:, 0]
        return (self.forward_tm(x.transpose(1, 2), m) * m.unsqueeze(-1)).transpose(1, 2)


class _Embedding(torch.autograd.Function):
    """embedding(ids) * scale (text_encoder.py:389) in one HIP launch; the weight gradient sums each
    token's rows in index order (csrc/embedding.hip) -- deterministic, where torch's embedding backward
    uses atomics -- so the whole train step is bit-reproducible run to run."""

    @staticmethod
    def forward(ctx, ids, weight, scale):
        N.require_device(ids, weight)
        ids_c = ids.reshape(-1).to(torch.int64).contiguous()
        w = weight.detach().to(torch.float32).contiguous()
        V, C = w.shape
        out = torch.empty(ids_c.numel(), C, dtype=torch.float32, device=w.device)
        with torch.cuda.device(w.device):
            N.check(N.lib().mtts_embedding_fwd(N.ptr(ids_c), N.ptr(w), ids_c.numel(), V, C, float(scale), N.ptr(out),
                                               N.stream_handle(w.device)), "mtts_embedding_fwd")
        ctx.save_for_backward(ids_c)
        ctx.shape, ctx.scale = (V, C), float(scale)
        return out.view(*ids.shape, C)

    @staticmethod
    def backward(ctx, g):
        (ids_c,) = ctx.saved_tensors
        V, C = ctx.shape
        gc = g.detach().to(torch.float32).reshape(-1, C).contiguous()
        dw = torch.empty(V, C, dtype=torch.float32, device=gc.device)
        # the weight gradient is this backward's only output: inside a Trainer step it runs on the gradient
        # deferral's side stream, beside the final weight-gradient flush (outputs allocated here, inputs kept)
        # (only when the weight takes the gradient: a dropped output's memory could be reused under the side
        # kernel; and the output is not kept alive -- AccumulateGrad must steal it, not copy it)
        side = O.param_grad_side_stream() if ctx.needs_input_grad[1] else None
        if side is not None:
            O.keep_for_side(ids_c, gc)
        st = side.cuda_stream if side is not None else N.stream_handle(gc.device)
        with torch.cuda.device(gc.device):
            N.check(N.lib().mtts_embedding_bwd(N.ptr(ids_c), N.ptr(gc), ids_c.numel(), V, C, ctx.scale, N.ptr(dw),
                                               st), "mtts_embedding_bwd")
        return None, dw, None


N.register("mtts_embedding_fwd", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                                ctypes.c_int32, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p])
N.register("mtts_embedding_bwd", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                                ctypes.c_int32, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p])


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
            self.prenet = None
        self.encoder = Encoder(self.channel_dim, encoder_params.filter_channels, encoder_params.n_heads,
                               encoder_params.n_layers, encoder_params.kernel_size, encoder_params.p_dropout)
        self.mean_projection = nn.Conv1d(self.channel_dim, self.feature_dim, 1)
        self.duration_predictor = DurationPredictor(self.channel_dim, duration_predictor_params.filter_channels_dp,
                                                    duration_predictor_params.kernel_size,
                                                    duration_predictor_params.p_dropout)

    def forward(self, text_input, text_lengths):
        """text_encoder.py:376-402 -> (mu [B, n_feats, T], logw [B, 1, T], x_mask [B, 1, T])."""
        with O.weight_pack_scope(self):
            # [B, T, C]: token-major already
            emb = _Embedding.apply(text_input, self.embedding.weight, math.sqrt(self.channel_dim))
            # sequence_mask(...).to(float) and the attention's -1e4 key bias in one launch
            m, key_bias = O.sequence_mask_f32(text_lengths, emb.size(1), key_bias=True)
            h = self.prenet.forward_tm(emb, m) if self.prenet is not None else emb
            h = self.encoder.forward_tm(h, m, key_bias)
            mu = O.linear_tm(h, self.mean_projection.weight, self.mean_projection.bias, in_scale=m, out_scale=m)
            logw = self.duration_predictor.forward_tm(h.detach(), m)
        return mu.transpose(1, 2), logw.transpose(1, 2), m.unsqueeze(1)
