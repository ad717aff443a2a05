"""Conditional flow matching: training loss and Euler sampler (drop-in for
matcha/models/components/flow_matching.py).

Reference: BaseConditionalFlowMatching flow_matching.py:12-151, ConditionalFlowMatching :154-189.
compute_loss keeps the reference's RNG order (t = rand([B,1,1]) then z = randn_like(x1), :130,:133),
its unmasked velocity target (:142) and its sum / (sum(mask) * n_feats) normalisation (:148-149).
Keyword-only ``t``/``z`` let parity tests inject the randomness.
"""
from __future__ import annotations

from abc import ABC

import torch
import torch.nn as nn

from matcha import _native as N
from matcha.models.components import _ops as O
from matcha.models.components.decoder import Decoder


class _FusedLosses(torch.autograd.Function):
    """CFM loss (flow_matching.py:145-149) and prior loss (matcha_tts.py:319-323) with their backward
    in three HIP launches (csrc/losses.hip: partials + finalize forward, one backward) instead of
    ~30 elementwise / reduction kernels.  u_pred token-major [B,T,C] (or None: no CFM term);
    mu_y [B,C,T] (or None: no prior term); x1 = y, z [B,C,T]; mask [B,T].  Returns two fp32 scalars."""

    @staticmethod
    def forward(ctx, u_pred, mu_y, x1, z, mask, sigma_min):
        N.require_device(x1, mask)
        f32 = lambda t: None if t is None else t.detach().to(torch.float32).contiguous()  # noqa: E731
        u_c, mu_c, x1_c, z_c, m_c = f32(u_pred), f32(mu_y), f32(x1), f32(z), f32(mask)
        B, C, T = x1_c.shape
        if u_c is not None and (u_c.shape != (B, T, C) or z_c is None or z_c.shape != x1_c.shape):
            raise ValueError("fused losses: u_pred must be [B, T, C] and z [B, C, T]")
        if mu_c is not None and mu_c.shape != x1_c.shape:
            raise ValueError("fused losses: mu_y must be [B, C, T]")
        if m_c.shape != (B, T):
            raise ValueError("fused losses: mask must be [B, T]")
        dev = x1_c.device
        out = torch.empty(3, dtype=torch.float32, device=dev)
        ws = torch.empty(max(int(N.lib().mtts_losses_workspace_size(B, T)), 4), dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            N.check(N.lib().mtts_losses_fwd(N.ptr(u_c), N.ptr(x1_c), N.ptr(z_c), N.ptr(x1_c), N.ptr(mu_c), N.ptr(m_c),
                                            B, C, T, float(sigma_min), N.ptr(out), N.ptr(ws), ws.numel(),
                                            N.stream_handle(dev)), "mtts_losses_fwd")
        ctx.save_for_backward(u_c, mu_c, x1_c, z_c, m_c, out)
        ctx.sigma = float(sigma_min)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_diff, g_prior):
        u_c, mu_c, x1_c, z_c, m_c, out = ctx.saved_tensors
        B, C, T = x1_c.shape
        need_u = ctx.needs_input_grad[0] and u_c is not None
        need_mu = ctx.needs_input_grad[1] and mu_c is not None
        du = torch.empty_like(u_c) if need_u else None
        dmu = torch.empty_like(mu_c) if need_mu else None
        gd = g_diff.detach().to(torch.float32).contiguous() if need_u else None
        gp = g_prior.detach().to(torch.float32).contiguous() if need_mu else None
        if need_u or need_mu:
            dev = x1_c.device
            with torch.cuda.device(dev):
                N.check(N.lib().mtts_losses_bwd(N.ptr(gd), N.ptr(gp), N.ptr(out), N.ptr(u_c), N.ptr(x1_c), N.ptr(z_c),
                                                N.ptr(x1_c), N.ptr(mu_c), N.ptr(m_c), B, C, T, ctx.sigma, N.ptr(du),
                                                N.ptr(dmu), N.stream_handle(dev)), "mtts_losses_bwd")
        return du, dmu, None, None, None, None


class _CfmPack(torch.autograd.Function):
    """phi_t = (1 - (1 - sigma) t) z + t x1 (flow_matching.py:138) packed with mu into the decoder's
    token-major input [B, T, 2C] (decoder.py:288) in one HIP pass (csrc/cfm_prep.hip); backward
    returns mu's gradient (x1 = y, z and t carry none, as in the reference)."""

    @staticmethod
    def forward(ctx, x1, z, t, mu, sigma_min):
        N.require_device(x1, z, t, mu)
        x1c, zc, muc = (v.detach().to(torch.float32).contiguous() for v in (x1, z, mu))
        tc = t.detach().to(torch.float32).reshape(-1).contiguous()
        B, C, T = x1c.shape
        if zc.shape != x1c.shape or muc.shape != x1c.shape or tc.numel() != B:
            raise ValueError("cfm pack: x1, z, mu must be [B, C, T] and t [B]")
        packed = torch.empty((B, T, 2 * C), dtype=torch.float32, device=x1c.device)
        with torch.cuda.device(x1c.device):
            N.check(N.lib().mtts_cfm_pack_fwd(N.ptr(x1c), N.ptr(zc), N.ptr(tc), N.ptr(muc), B, C, T, float(sigma_min),
                                              N.ptr(packed), N.stream_handle(x1c.device)), "mtts_cfm_pack_fwd")
        ctx.shape = (B, C, T)
        return packed

    @staticmethod
    def backward(ctx, d_packed):
        if not ctx.needs_input_grad[3]:
            return None, None, None, None, None
        B, C, T = ctx.shape
        dp = d_packed.detach().to(torch.float32).contiguous()
        d_mu = torch.empty((B, C, T), dtype=torch.float32, device=dp.device)
        with torch.cuda.device(dp.device):
            N.check(N.lib().mtts_cfm_pack_bwd(N.ptr(dp), B, C, T, N.ptr(d_mu), N.stream_handle(dp.device)),
                    "mtts_cfm_pack_bwd")
            # the decoder's backward is complete: its queued weight gradients overlap the encoder's backward
            O.flush_deferred_side()
        return None, None, None, d_mu, None


def fused_losses(u_pred, mu_y, x1, z, mask, sigma_min):
    """(diff_loss, prior_loss); see _FusedLosses.  mask [B, 1, T] or [B, T]."""
    if mask.dim() == 3:
        mask = mask[:, 0]
    return _FusedLosses.apply(u_pred, mu_y, x1, z, mask, sigma_min)


class BaseConditionalFlowMatching(nn.Module, ABC):
    def __init__(self, n_feats, cfm_params, n_spks=1, spk_emb_dim=128):
        super().__init__()
        self.n_feats = n_feats
        self.n_spks = n_spks
        self.spk_emb_dim = spk_emb_dim
        self.solver = getattr(cfm_params, "solver", "euler")
        self.sigma_min = getattr(cfm_params, "sigma_min", 1e-4)
        self.estimator = None

    @torch.inference_mode()
    def forward(self, mu, mask, n_timesteps, temperature=1.0, spks=None, cond=None, *, z=None):
        """flow_matching.py:42-65: Euler integration of the learned velocity from N(0, T^2).
        ``z`` (keyword-only) injects the initial noise for parity tests."""
        if z is None:
            z = torch.randn_like(mu) * temperature
        t_span = torch.linspace(0, 1, n_timesteps + 1, device=mu.device)
        return self.solve_ode_euler(z, t_span, mu, mask, spks, cond)

    # the whole Euler solve of one (shape, n_timesteps) is captured once into a HIP graph and replayed:
    # n_timesteps decoder forwards (~70 kernels each) become one graph launch.  Bounded cache.
    graph_ode: bool = True
    _GRAPH_CACHE_MAX = 8

    def solve_ode_euler(self, x, t_span, mu, mask, spks, cond):
        """flow_matching.py:67-104 (same t/dt recurrence).  The velocity field runs token-major on the
        HIP kernels (Decoder.forward_tm); the state stays [B, T, C] across the steps and is transposed
        back once at the end."""
        if self.graph_ode and x.is_cuda and not torch.cuda.is_current_stream_capturing():
            return self._solve_graph(x, t_span, mu, mask)
        return self._solve_eager(x, t_span, mu, mask)

    def _solve_graph(self, x, t_span, mu, mask):
        cache = self.__dict__.setdefault("_ode_graphs", {})
        key = (tuple(x.shape), tuple(mu.shape), t_span.numel(), x.dtype, x.device,
               torch.is_autocast_enabled("cuda"), torch.get_autocast_dtype("cuda"))
        ent = cache.get(key)
        if ent is None:
            if len(cache) >= self._GRAPH_CACHE_MAX:
                cache.pop(next(iter(cache)))
            sx, smu, sm, st = x.clone(), mu.clone(), mask.clone(), t_span.clone()
            cur = torch.cuda.current_stream(x.device)
            side = torch.cuda.Stream(x.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):  # warm-up: lazy loads, pack plans, allocator pools
                self._solve_eager(sx, st, smu, sm)
            cur.wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = self._solve_eager(sx, st, smu, sm)
            ent = cache[key] = (g, sx, smu, sm, st, out)
        g, sx, smu, sm, st, out = ent
        sx.copy_(x)
        smu.copy_(mu)
        sm.copy_(mask)
        st.copy_(t_span)
        g.replay()
        return out.clone()

    def _solve_eager(self, x, t_span, mu, mask):
        t = t_span[0]
        dt = t_span[1] - t_span[0]
        xt = x.transpose(1, 2).contiguous()
        mu_t = mu.transpose(1, 2).contiguous()
        m = mask[:, 0].contiguous()
        for step in range(1, len(t_span)):
            xt = xt + dt * self.estimator.forward_tm(xt, m, mu_t, t.expand(x.shape[0]))
            t = t + dt
            if step < len(t_span) - 1:
                dt = t_span[step + 1] - t
        return xt.transpose(1, 2)

    def compute_loss(self, x1, mask, mu, spks=None, cond=None, *, t=None, z=None):
        """Returns (loss, phi_t).  x1/mu [B, n_feats, T], mask [B, 1, T]."""
        loss, _, phi_t = self.compute_loss_and_prior(x1, mask, mu, None, t=t, z=z)
        return loss, phi_t

    def compute_loss_and_prior(self, x1, mask, mu, prior_mu, *, t=None, z=None, segments=1):
        """compute_loss plus, when prior_mu is given, MatchaTTS's prior loss on (x1, prior_mu) -- both
        in one fused pass over the tensors (csrc/losses.hip).  Returns (diff_loss, prior_loss, phi_t).
        segments = n > 1: the losses of each of n equal micro-batches stacked along dim 0 ([n] tensors)."""
        b = mu.shape[0]
        if t is None:
            t = torch.rand([b, 1, 1], device=mu.device, dtype=mu.dtype)
        if z is None:
            z = torch.randn_like(x1)
        s = self.sigma_min
        # phi_t (:139) packed with mu into the decoder's token-major input in one launch
        packed = _CfmPack.apply(x1, z, t, mu, s)
        phi_t = packed[..., : x1.shape[1]].transpose(1, 2)
        u_pred = self.estimator.forward_tm_packed(packed, mask[:, 0], t.reshape(b))
        # sum((u_pred - u)^2) / (sum(mask) * n_feats) and the prior loss, fused (flow_matching.py:145-149)
        if segments > 1:
            bs = b // segments
            sl = [slice(i * bs, (i + 1) * bs) for i in range(segments)]
            parts = [fused_losses(u_pred[q], prior_mu[q] if prior_mu is not None else None, x1[q], z[q], mask[q], s)
                     for q in sl]
            loss = torch.stack([lp[0] for lp in parts])
            prior = torch.stack([lp[1] for lp in parts]) if prior_mu is not None else None
            return loss, prior, phi_t
        loss, prior = fused_losses(u_pred, prior_mu, x1, z, mask, s)
        return loss, prior, phi_t


class ConditionalFlowMatching(BaseConditionalFlowMatching):
    def __init__(self, in_channels, out_channel, cfm_params, decoder_params, n_spks=1, spk_emb_dim=64):
        super().__init__(n_feats=in_channels, cfm_params=cfm_params, n_spks=n_spks, spk_emb_dim=spk_emb_dim)
        if n_spks > 1:
            in_channels = in_channels + spk_emb_dim
        self.estimator = Decoder(in_channels=in_channels, out_channels=out_channel, **decoder_params)


CFM = ConditionalFlowMatching
