"""Token-major ([B, T, C], C contiguous) device operators of the CFM decoder.

The reference runs the decoder channel-major ([B, C, T]) and rearranges to [B, T, C] around every
transformer block (decoder.py:298-306, 324-332, 345-353).  Here activations stay token-major for the
whole U-Net: a k-tap Conv1d is an implicit GEMM over K = k*C_in with rows = tokens, the transformer
GEMMs need no transposes, and the reference's rearranges disappear.

Each operator below is the unit a HIP kernel replaces (csrc/decoder_*.hip via include/mtts_decoder.h);
`KERNELS` records which operators currently run in libmtts_hip.so.  Operators not yet moved run as
PyTorch-ROCm device ops; none of them runs on the host.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

KERNELS: dict[str, str] = {}


def _cm(x: torch.Tensor) -> torch.Tensor:  # token-major -> channel-major view
    return x.transpose(1, 2)


def conv_tm(x, weight, bias, mask=None, stride: int = 1, padding: int | None = None):
    """y = Conv1d(x * mask) in token-major layout.  x [B,T,Cin], weight [Cout,Cin,k] (nn.Conv1d
    layout), mask [B,T] or None.  decoder.py:59,65,78,85,95,192,239,248,251."""
    k = weight.shape[-1]
    if padding is None:
        padding = k // 2
    if mask is not None:
        x = x * mask.unsqueeze(-1)
    return F.conv1d(_cm(x), weight, bias, stride=stride, padding=padding).transpose(1, 2)


def conv_transpose_tm(x, weight, bias, mask=None):
    """ConvTranspose1d(k=4, s=2, p=1) of x * mask; weight [Cin,Cout,4].  decoder.py:112-116."""
    if mask is not None:
        x = x * mask.unsqueeze(-1)
    return F.conv_transpose1d(_cm(x), weight, bias, stride=2, padding=1).transpose(1, 2)


def group_norm_mish_tm(h, gamma, beta, groups: int, mask, add=None, eps: float = 1e-5):
    """mish(GroupNorm(h)) * mask (+ add[b, c]).  Block1D tail (decoder.py:58-66) with the ResNet
    time-embedding injection (decoder.py:82-83) fused.  GN statistics span the full padded length,
    exactly like the reference."""
    y = F.mish(F.group_norm(_cm(h), groups, gamma, beta, eps)).transpose(1, 2) * mask.unsqueeze(-1)
    if add is not None:
        y = y + add.unsqueeze(1)
    return y


def layer_norm_tm(h, weight, bias, eps: float = 1e-5):
    return F.layer_norm(h, (h.shape[-1],), weight, bias, eps)


def linear_tm(x, weight, bias=None, act: str | None = None, residual=None):
    """x @ W^T + b, optional erf-GELU epilogue or residual add (transformer.py:155-156,174-180,
    diffusers to_out)."""
    y = F.linear(x, weight, bias)
    if act == "gelu":
        y = F.gelu(y)
    if residual is not None:
        y = y + residual
    return y


def attention_tm(q, k, v, key_bias, heads: int):
    """softmax(q k^T / sqrt(d) + key_bias[b, key]) v per head.  q/k/v [B,T,H*d], key_bias [B,T]:
    the reference's float 0/1 mask is ADDED to the scores (diffusers AttnProcessor2_0 +
    prepare_attention_mask), so padded keys are down-weighted, not removed."""
    B, T, C = q.shape
    d = C // heads
    qh = q.view(B, T, heads, d).transpose(1, 2)
    kh = k.view(B, T, heads, d).transpose(1, 2)
    vh = v.view(B, T, heads, d).transpose(1, 2)
    bias = key_bias.to(q.dtype)[:, None, None, :].expand(B, heads, T, T)
    o = F.scaled_dot_product_attention(qh, kh, vh, attn_mask=bias, scale=1.0 / math.sqrt(d))
    return o.transpose(1, 2).reshape(B, T, C)
