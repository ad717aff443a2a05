"""CFM velocity estimator: 1-D U-Net of ResNet + transformer blocks (drop-in for
matcha/models/components/decoder.py).

Same constructor, same module tree and parameter names as the reference (decoder.py:118-253), same
forward signature ``forward(x, mask, mu, t, cond=None)`` with channel-major [B, C, T] in/out.
Internally the activations are token-major [B, T, C] from the input pack to the final projection
(see _ops.py); the reference's semantics are kept exactly, including its padding-dependent quirks:
GroupNorm statistics over the full padded length, the ResNet residual not re-masked (:85), the
half-resolution mask as a prefix slice (:311-316), nearest interpolation for odd lengths (:338-339,
:361-364), and the float 0/1 attention mask used as an additive bias.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from matcha import _native as N
from matcha.models.components import _ops as O
from matcha.models.components.transformer import BasicTransformerBlock

# MTTS_RESNET_DX_LINK=0: autograd sums Resnet1D's two input gradients (A/B switch; the sum is the same)
_DX_LINK = os.environ.get("MTTS_RESNET_DX_LINK", "1") != "0"
# MTTS_RESNET_BF16_STORE=0: bf16-mixed keeps the ResNet blocks' conv outputs / GroupNorm outputs in fp32
# (precision-budget switch, tools/r3/precision_budget.py)
_RESNET16 = os.environ.get("MTTS_RESNET_BF16_STORE", "1") != "0"


class SinusoidalPosEmb(nn.Module):
    """decoder.py:8-31: t -> [sin(1000 t f_k), cos(1000 t f_k)], f_k = exp(-k ln(1e4)/(dim/2-1))."""

    def __init__(self, dim):
        super().__init__()
        assert dim % 2 == 0, "SinusoidalPosEmb needs an even dimension"
        self.dim = dim

    def forward(self, x, scale=1000):
        if x.ndim < 1:
            x = x.unsqueeze(0)
        # one HIP launch (csrc/cfm_prep.hip) for arange / exp / mul / sin / cos / cat, torch's fp32 order
        N.require_device(x)
        xc = x.detach().float().reshape(-1).contiguous()
        out = torch.empty((xc.numel(), self.dim), dtype=torch.float32, device=x.device)
        with torch.cuda.device(x.device):
            N.check(N.lib().mtts_time_embedding(N.ptr(xc), xc.numel(), self.dim, float(scale), N.ptr(out),
                                                N.stream_handle(x.device)), "mtts_time_embedding")
        return out


class TimeStepEmbeddingNet(nn.Module):
    """decoder.py:33-49: Linear -> SiLU -> Linear on [B, in]."""

    def __init__(self, in_channels, time_embed_dim):
        super().__init__()
        self.linear_1 = nn.Linear(in_channels, time_embed_dim)
        self.act = nn.SiLU()
        self.linear_2 = nn.Linear(time_embed_dim, time_embed_dim)

    def forward(self, sample):
        return self.linear_2(self.act(self.linear_1(sample)))


class Block1D(nn.Module):
    """decoder.py:51-66: mish(GN(conv3(x*m))) * m  -- token-major, GN+Mish+mask fused."""

    def __init__(self, in_channels, out_channels, kernel_size=3, padding=1, groups=8):
        super().__init__()
        self.block = nn.Sequential(
            nn.Conv1d(in_channels, out_channels, kernel_size, padding=padding),
            nn.GroupNorm(groups, out_channels),
            nn.Mish(),
        )

    def forward_tm(self, x, mask, add=None, out_bf16=False, dx_link=None):
        """bf16-mixed: the conv output (read only by the GroupNorm) is stored as bf16, and so is the
        result when out_bf16 (its only consumer is the next conv's GEMM) -- as autocast would hold them.
        dx_link: the conv takes the other consumer's input gradient into its dgrad (O.GradLink)."""
        conv, gn = self.block[0], self.block[1]
        h = O.conv_tm(x, conv.weight, conv.bias, mask, padding=conv.padding[0], out_bf16=_RESNET16,
                      dx_link=dx_link, dx_link_role="take" if dx_link is not None else None)
        return O.group_norm_mish_tm(h, gn.weight, gn.bias, gn.num_groups, mask, add, gn.eps,
                                    out_bf16=out_bf16 and _RESNET16)

    def forward(self, x, mask):  # channel-major API of the reference
        return self.forward_tm(x.transpose(1, 2), mask[:, 0]).transpose(1, 2)


class Resnet1D(nn.Module):
    """decoder.py:68-86: block2(block1(x) + mlp(t)) + res_conv(x*m); the result is not re-masked."""

    def __init__(self, in_channels, out_channels, time_emb_dim, kernel_size=3, padding=1, groups=8):
        super().__init__()
        self.mlp = nn.Sequential(nn.Mish(), nn.Linear(time_emb_dim, out_channels))
        self.block1 = Block1D(in_channels, out_channels, kernel_size, padding, groups)
        self.block2 = Block1D(out_channels, out_channels, kernel_size, padding, groups)
        self.res_conv = nn.Conv1d(in_channels, out_channels, 1)

    def forward_tm(self, x, mask, time_emb, tproj=None):
        """tproj: this block's mlp(time_emb) when the caller computed every block's at once."""
        if tproj is None:
            with torch.autocast("cuda", enabled=False):  # [B, C] time projection, fp32
                tproj = self.mlp(time_emb.float())
        # x feeds block1's conv and res_conv: res_conv's input gradient is added in block1's dgrad epilogue
        link = O.GradLink() if _DX_LINK and x.requires_grad and torch.is_grad_enabled() else None
        h = self.block1.forward_tm(x, mask, add=tproj, out_bf16=True, dx_link=link)
        h = self.block2.forward_tm(h, mask)  # fp32: the residual of res_conv's epilogue
        # res_conv(x*m) + h with the add in the GEMM epilogue ((acc + bias) + h, torch's order)
        return O.conv_tm(x, self.res_conv.weight, self.res_conv.bias, mask, padding=0, residual=h,
                         dx_link=link, dx_link_role="give" if link is not None else None)

    def forward(self, x, mask, time_emb):
        return self.forward_tm(x.transpose(1, 2), mask[:, 0], time_emb).transpose(1, 2)


class Downsample1D(nn.Module):
    """decoder.py:88-98: Conv1d(k3, s2, p1) -> ceil(T/2) frames."""

    def __init__(self, dim):
        super().__init__()
        self.conv = nn.Conv1d(dim, dim, kernel_size=3, stride=2, padding=1)

    def forward_tm(self, x, mask, dx_link=None):
        return O.conv_tm(x, self.conv.weight, self.conv.bias, mask, stride=2, padding=1, dx_link=dx_link,
                         dx_link_role="take" if dx_link is not None else None)

    def forward(self, x):
        return self.conv(x)


class Upsample1D(nn.Module):
    """decoder.py:100-116: ConvTranspose1d(k4, s2, p1) -> 2T frames."""

    def __init__(self, channels, out_channels=None):
        super().__init__()
        self.channels = channels
        self.out_channels = out_channels or channels
        self.conv = nn.ConvTranspose1d(channels, self.out_channels, 4, 2, 1)

    def forward_tm(self, x, mask):
        return O.conv_transpose_tm(x, self.conv.weight, self.conv.bias, mask)

    def forward(self, inputs):
        assert inputs.shape[1] == self.channels
        return self.conv(inputs)


def _conv_tm(mod: nn.Conv1d, x, mask, dx_link=None):
    return O.conv_tm(x, mod.weight, mod.bias, mask, stride=mod.stride[0], padding=mod.padding[0], dx_link=dx_link,
                     dx_link_role="take" if dx_link is not None else None)


class Decoder(nn.Module):
    """decoder.py:118-371.  channels=(256,256), 1 transformer per level, 2 mid blocks, 4 heads x 64."""

    def __init__(self, in_channels, out_channels, channels=(256, 256), dropout=0.05, attention_head_dim=64,
                 n_blocks=1, num_mid_blocks=2, num_heads=4):
        super().__init__()
        channels = tuple(channels)
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.time_embeddings = SinusoidalPosEmb(dim=in_channels)
        time_embed_dim = channels[0] * 4
        self.time_mlp = TimeStepEmbeddingNet(in_channels, time_embed_dim)

        def tblocks(dim):
            return nn.ModuleList([
                BasicTransformerBlock(dim=dim, num_attention_heads=num_heads, attention_head_dim=attention_head_dim,
                                      dropout=dropout, activation_fn="gelu")
                for _ in range(n_blocks)])

        self.Downsampling_Blocks = nn.ModuleList([])
        self.Mid_Blocks = nn.ModuleList([])
        self.Upsampling_Blocks = nn.ModuleList([])
        out_c = in_channels
        for i, c in enumerate(channels):
            in_c, out_c = out_c, c
            last = i == len(channels) - 1
            down = nn.Conv1d(out_c, out_c, kernel_size=3, padding=1) if last else Downsample1D(out_c)
            self.Downsampling_Blocks.append(nn.ModuleList([Resnet1D(in_c, out_c, time_embed_dim), tblocks(out_c), down]))
        for _ in range(num_mid_blocks):
            self.Mid_Blocks.append(nn.ModuleList([Resnet1D(channels[-1], channels[-1], time_embed_dim),
                                                  tblocks(channels[-1])]))
        rev = channels[::-1] + (channels[0],)
        for i in range(len(rev) - 1):
            last = i == len(rev) - 2
            up = nn.Conv1d(rev[i + 1], rev[i + 1], kernel_size=3, padding=1) if last else Upsample1D(rev[i + 1])
            self.Upsampling_Blocks.append(nn.ModuleList([Resnet1D(2 * rev[i], rev[i + 1], time_embed_dim),
                                                         tblocks(rev[i + 1]), up]))
        self.final_conv = nn.Conv1d(channels[0], channels[0], kernel_size=3, padding=1)
        self.final_norm = nn.GroupNorm(8, channels[0])
        self.final_act = nn.Mish()
        self.final_proj = nn.Conv1d(channels[0], self.out_channels, kernel_size=1)
        self.initialize_weights()

    def initialize_weights(self):
        """decoder.py:255-268 (kaiming-normal convs/linears, zero biases, unit GroupNorm)."""
        for m in self.modules():
            if isinstance(m, (nn.Conv1d, nn.Linear)):
                nn.init.kaiming_normal_(m.weight, nonlinearity="relu")
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.GroupNorm):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    @staticmethod
    def _transformers(blocks, x, mask):
        for blk in blocks:
            x = blk.forward_tm(x, mask)
        return x

    def forward_tm(self, x, mask, mu, t):
        """x, mu: [B, T, C] token-major; mask [B, T]; t [B] -> [B, T, out] token-major.
        GEMMs run bf16 MFMA inside a bf16 autocast region (fp32 accumulate, fp32 activations), exact
        fp32 MFMA otherwise; everything else here is fp32."""
        prec_bf16 = torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
        with torch.autocast("cuda", enabled=False):
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=prec_bf16), O.weight_pack_scope(self):
                return self._forward_tm(x.float(), mask.float(), mu.float(), t.float())

    def forward_tm_packed(self, h, mask, t):
        """forward_tm on the already packed input h = [x | mu] [B, T, 2C] (CFM's fused pack)."""
        prec_bf16 = torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
        with torch.autocast("cuda", enabled=False):
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=prec_bf16), O.weight_pack_scope(self):
                return self._forward_tm(None, mask.float(), None, t.float(), packed=h)

    def _resnets(self):
        return ([r for r, *_ in self.Downsampling_Blocks] + [r for r, _ in self.Mid_Blocks]
                + [r for r, *_ in self.Upsampling_Blocks])

    def prefetch(self, t, side):
        """Launches, on `side` (already ordered after the current stream), what this decoder's next forward
        for CFM time t needs and nothing else produces: its weight packs and the time path (embedding +
        time MLP forward).  Outputs are allocated on the current stream; forward waits for `side` where it
        uses them (weight_pack_scope, _time_path) -- a Trainer step runs them beside the text encoder."""
        O.prefetch_packs(self, side)
        resnets = self._resnets()
        with torch.autocast("cuda", enabled=False):
            tt = t.detach().float().reshape(-1).contiguous()
            e = torch.empty((tt.numel(), self.time_embeddings.dim), dtype=torch.float32, device=tt.device)
            O.keep_for_side(tt, e)
            with torch.cuda.device(tt.device):
                N.check(N.lib().mtts_time_embedding(N.ptr(tt), tt.numel(), self.time_embeddings.dim, 1000.0, N.ptr(e),
                                                    side.cuda_stream), "mtts_time_embedding")
            pre = O.time_mlp_ahead(e, self.time_mlp.linear_1, self.time_mlp.linear_2, [r.mlp[1] for r in resnets], side)
        self.__dict__["_mtts_time_pre"] = (tt.data_ptr(), tt.numel(), e, pre, side)

    def _time_path(self, t):
        """temb = time_mlp(SinusoidalPosEmb(t)) (decoder.py:33-49, :285-286) and every Resnet1D's
        mlp(temb) = Linear(Mish(temb)) (:80-81), fp32 as the reference keeps it, in 1 + 3 HIP launches (one
        more per further 8 blocks)
        (csrc/cfm_prep.hip, csrc/time_mlp.hip) -- or prefetched for this t (prefetch); backward 5.
        Returns (temb, {id(resnet): tp})."""
        resnets = self._resnets()
        pre = self.__dict__.pop("_mtts_time_pre", None)
        with torch.autocast("cuda", enabled=False):
            tt = t.detach().float().reshape(-1)
            if pre is not None and pre[0] == tt.data_ptr() and pre[1] == tt.numel():
                torch.cuda.current_stream(tt.device).wait_stream(pre[4])
                temb, tps = O.time_mlp(pre[2], self.time_mlp.linear_1, self.time_mlp.linear_2,
                                       [r.mlp[1] for r in resnets], pre=pre[3])
            else:
                e = self.time_embeddings(t)
                temb, tps = O.time_mlp(e, self.time_mlp.linear_1, self.time_mlp.linear_2, [r.mlp[1] for r in resnets])
        return temb, dict(zip(map(id, resnets), tps))

    def _forward_tm(self, x, mask, mu, t, packed=None):
        temb, tps = self._time_path(t)  # [B, 1024] time MLP + every block's projection, fp32
        h = torch.cat([x, mu], dim=-1) if packed is None else packed  # einops pack "b * t" on channels (:288)
        skips, masks = [], [mask]
        for resnet, tfs, down in self.Downsampling_Blocks:
            m = masks[-1]
            h = self._transformers(tfs, resnet.forward_tm(h, m, temb, tps[id(resnet)]), m)
            # the skip feeds this level's down conv and (later) the up path's concat: the concat hands its
            # slice of the gradient to the down conv's dgrad epilogue (GradLink)
            link = O.GradLink() if _DX_LINK and h.requires_grad and torch.is_grad_enabled() else None
            skips.append((h, link))
            if isinstance(down, Downsample1D):
                h = down.forward_tm(h, m, dx_link=link)
                # prefix slice (:311-316), made contiguous once (every op of the level reads it)
                masks.append(m[:, : (m.shape[-1] + 1) // 2].contiguous())
            else:
                h = _conv_tm(down, h, m, dx_link=link)
                masks.append(m)
        masks = masks[:-1]
        m = masks[-1]
        for resnet, tfs in self.Mid_Blocks:
            h = self._transformers(tfs, resnet.forward_tm(h, m, temb, tps[id(resnet)]), m)
        n_up = len(self.Upsampling_Blocks)
        for i_up, (resnet, tfs, up) in enumerate(self.Upsampling_Blocks):
            m = masks.pop()
            skip, link = skips.pop()
            if h.shape[1] != skip.shape[1]:  # odd T: nearest to the skip length (:338-339)
                h = F.interpolate(h.transpose(1, 2), size=skip.shape[1], mode="nearest").transpose(1, 2)
            h = O.cat_skip_tm(h, skip, link)  # einops pack on channels (:341)
            h = self._transformers(tfs, resnet.forward_tm(h, m, temb, tps[id(resnet)]), m)
            if isinstance(up, Upsample1D):
                h = up.forward_tm(h, m)
                new = m.shape[-1] * 2
            else:
                h = _conv_tm(up, h, m)
                new = h.shape[1]
            if i_up + 1 < n_up:  # the next block pops its own mask: this one is only read by the head
                continue
            if new > m.shape[-1]:
                m = F.interpolate(m.unsqueeze(1), size=new, mode="nearest")[:, 0]
            else:
                m = m[:, :new].contiguous()
        fc = self.final_conv
        h = O.conv_tm(h, fc.weight, fc.bias, m, stride=fc.stride[0], padding=fc.padding[0], out_bf16=_RESNET16)
        h = O.group_norm_mish_tm(h, self.final_norm.weight, self.final_norm.bias, self.final_norm.num_groups,
                                 None, None, self.final_norm.eps, out_bf16=_RESNET16)  # no mask after the Mish (:366-368)
        return O.conv_tm(h, self.final_proj.weight, self.final_proj.bias, m, padding=0, out_scale=mask)

    def forward(self, x, mask, mu, t, cond=None):
        """Reference signature: x, mu [B, C, T]; mask [B, 1, T]; t [B] -> [B, out, T]."""
        out = self.forward_tm(x.transpose(1, 2), mask[:, 0], mu.transpose(1, 2), t)
        return out.transpose(1, 2)
