"""Decoder transformer block (drop-in for matcha/models/components/transformer.py, diffusers branch).

Reference: BasicTransformerBlock transformer.py:191-370 (pre-LN: h += Attn(LN1(h)); h += FF(LN3(h))),
FeedForward :105-188 (diffusers GELU(dim, 4*dim) = Linear + erf-GELU, Dropout, Linear), and diffusers
0.25 Attention / AttnProcessor2_0 (to_q/k/v without bias, to_out = [Linear, Dropout], SDPA with the
float 0/1 mask as an additive bias).  Module tree and parameter names match the reference
(norm1, attn1.to_q/to_k/to_v/to_out.0, norm3, ff.net.0.proj, ff.net.2).

Token-major forward (``forward_tm``): the q/k/v projections run as ONE GEMM against the concatenated
[3C, C] weight, the residual adds are fused into the to_out and ff.net.2 GEMM epilogues.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn

from matcha.models.components import _ops as O

# MTTS_PRELN_FUSED=0: BasicTransformerBlock.forward_tm runs op by op (A/B measurements)
_PRELN_FUSED = os.environ.get("MTTS_PRELN_FUSED", "1") != "0"


class GELU(nn.Module):
    """diffusers GELU(dim_in, dim_out, approximate='none'): Linear then erf-GELU."""

    def __init__(self, dim_in, dim_out, approximate="none", bias=True):
        super().__init__()
        if approximate != "none":
            raise NotImplementedError("the Matcha decoder uses the erf GELU only")
        self.proj = nn.Linear(dim_in, dim_out, bias=bias)

    def forward(self, x):
        return torch.nn.functional.gelu(self.proj(x))


class FeedForward(nn.Module):
    """transformer.py:105-188 with activation_fn='gelu' (the only one the decoder builds)."""

    def __init__(self, dim, dim_out=None, mult=4, dropout=0.0, activation_fn="gelu", final_dropout=False):
        super().__init__()
        if activation_fn != "gelu":
            raise NotImplementedError("the Matcha decoder builds FeedForward(activation_fn='gelu') only")
        inner = int(dim * mult)
        dim_out = dim_out if dim_out is not None else dim
        self.net = nn.ModuleList([GELU(dim, inner), nn.Dropout(dropout), nn.Linear(inner, dim_out)])
        if final_dropout:
            self.net.append(nn.Dropout(dropout))

    def forward_tm(self, x, residual=None):
        """residual + Linear2(Dropout(GELU(Linear1(x)))) as one fused op (GELU, dropout and the
        residual live in the GEMM epilogues)."""
        if len(self.net) > 3:
            raise NotImplementedError("final_dropout is not used by the Matcha decoder")
        p = self.net[1].p if self.training else 0.0
        proj, out = self.net[0].proj, self.net[2]
        return O.ff_tm(x, proj.weight, proj.bias, out.weight, out.bias, residual=residual, dropout_p=p)

    def forward(self, hidden_states):
        return self.forward_tm(hidden_states)


class Attention(nn.Module):
    """diffusers 0.25 Attention(query_dim, heads, dim_head, dropout, bias=False) self-attention."""

    def __init__(self, query_dim, heads=8, dim_head=64, dropout=0.0, bias=False, out_bias=True, **kw):
        super().__init__()
        inner = heads * dim_head
        self.heads = heads
        self.to_q = nn.Linear(query_dim, inner, bias=bias)
        self.to_k = nn.Linear(query_dim, inner, bias=bias)
        self.to_v = nn.Linear(query_dim, inner, bias=bias)
        self.to_out = nn.ModuleList([nn.Linear(inner, query_dim, bias=out_bias), nn.Dropout(dropout)])

    def qkv_weight(self):
        return torch.cat([self.to_q.weight, self.to_k.weight, self.to_v.weight], dim=0)

    def forward_tm(self, h, key_bias, residual=None):
        qkv = O.linear_tm(h, (self.to_q.weight, self.to_k.weight, self.to_v.weight), None)  # [B,T,3C] q|k|v
        o = O.attention_tm(qkv, key_bias, self.heads)
        p = self.to_out[1].p if self.training else 0.0
        return O.linear_tm(o, self.to_out[0].weight, self.to_out[0].bias, residual=residual, dropout_p=p)

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None, **kw):
        if encoder_hidden_states is not None:
            raise NotImplementedError("the decoder uses self-attention only")
        return self.forward_tm(hidden_states, attention_mask)


class BasicTransformerBlock(nn.Module):
    """transformer.py:191-370 (norm_type='layer_norm', no cross-attention, no ada-norm)."""

    def __init__(self, dim: int, num_attention_heads: int, attention_head_dim: int, dropout=0.0,
                 cross_attention_dim: Optional[int] = None, activation_fn: str = "geglu",
                 num_embeds_ada_norm: Optional[int] = None, attention_bias: bool = False,
                 only_cross_attention: bool = False, double_self_attention: bool = False,
                 upcast_attention: bool = False, norm_elementwise_affine: bool = True,
                 norm_type: str = "layer_norm", final_dropout: bool = False):
        super().__init__()
        if cross_attention_dim is not None or double_self_attention or num_embeds_ada_norm is not None:
            raise NotImplementedError("only the decoder's self-attention layer_norm block is built")
        self.norm1 = nn.LayerNorm(dim, elementwise_affine=norm_elementwise_affine)
        self.attn1 = Attention(dim, heads=num_attention_heads, dim_head=attention_head_dim, dropout=dropout,
                               bias=attention_bias)
        self.norm2 = None
        self.attn2 = None
        self.norm3 = nn.LayerNorm(dim, elementwise_affine=norm_elementwise_affine)
        self.ff = FeedForward(dim, dropout=dropout, activation_fn=activation_fn, final_dropout=final_dropout)

    def forward_tm(self, h, key_bias):
        """h [B, T, C]; key_bias [B, T] (the reference's float mask).  Each pre-LN residual sub-block is
        one fused op (components/_ops.py preln_attention_tm / preln_ff_tm)."""
        a, ff = self.attn1, self.ff
        if not _PRELN_FUSED:  # op-by-op composition (A/B measurements)
            n = O.layer_norm_tm(h, self.norm1.weight, self.norm1.bias, self.norm1.eps)
            h = a.forward_tm(n, key_bias, residual=h)
            n = O.layer_norm_tm(h, self.norm3.weight, self.norm3.bias, self.norm3.eps)
            return ff.forward_tm(n, residual=h)
        h = O.preln_attention_tm(h, self.norm1.weight, self.norm1.bias, self.norm1.eps, key_bias, a.heads,
                                 a.to_q.weight, a.to_k.weight, a.to_v.weight, a.to_out[0].weight, a.to_out[0].bias,
                                 dropout_p=a.to_out[1].p if self.training else 0.0)
        if len(ff.net) > 3:
            raise NotImplementedError("final_dropout is not used by the Matcha decoder")
        return O.preln_ff_tm(h, self.norm3.weight, self.norm3.bias, self.norm3.eps, ff.net[0].proj.weight,
                             ff.net[0].proj.bias, ff.net[2].weight, ff.net[2].bias,
                             dropout_p=ff.net[1].p if self.training else 0.0)

    def forward(self, hidden_states, attention_mask=None, encoder_hidden_states=None,
                encoder_attention_mask=None, timestep=None, cross_attention_kwargs=None, class_labels=None):
        if attention_mask is None:
            attention_mask = torch.zeros(hidden_states.shape[:2], device=hidden_states.device,
                                         dtype=hidden_states.dtype)
        return self.forward_tm(hidden_states, attention_mask)
