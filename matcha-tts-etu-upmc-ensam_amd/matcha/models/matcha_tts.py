"""Matcha-TTS model (drop-in for matcha/models/matcha_tts.py).

Reference: MatchaTTS matcha_tts.py:29-325 (config init :74-102, simple-params init :104-176, synthesise :178-245, forward :247-325).
The train-step forward keeps the reference's order and arithmetic; the monotonic alignment runs on
the GPU (matcha.utils.monotonic_align.maximum_path -> csrc/mas.hip) instead of the reference's
device->host->device Cython round trip, so the step never synchronises with the host.  The log-prior
lattice is computed in fp32 with autocast disabled: maximum_path is bit-exact only on the identical
fp32 lattice.
"""
from __future__ import annotations

import datetime as dt
import math
import os
import random
from types import SimpleNamespace

import torch

import matcha.utils.monotonic_align as monotonic_align
from matcha.models.baselightningmodule import BaseLightningClass
from matcha.models.components import _ops as O
from matcha.models.components.flow_matching import ConditionalFlowMatching as CFM
from matcha.models.components.text_encoder import TextEncoder
from matcha.utils.model import denormalize, fix_len_compatibility, generate_path, sequence_mask

# MTTS_PREFETCH=0: the decoder's weight packs and time path run in place instead of ahead on the side stream
_PREFETCH = os.environ.get("MTTS_PREFETCH", "1") != "0"


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


class MatchaTTS(BaseLightningClass):
    # text encoder precision inside a bf16-mixed region (see forward): "bf16" (autocast's), "fp32fwd" (the
    # forward on the exact-fp32 MFMA with fp32 weights -- 32-true's forward arithmetic --, backward bf16: the
    # parity policy since round 4), "bf16x3" (forward GEMMs as split bf16 operands A_hi W_hi + A_hi W_lo +
    # A_lo W_hi and an fp32 attention forward, backward bf16: ~16 significant bits, left an alignment
    # near-tie flipped), "fp32" (exact fp32 MFMA forward and backward)
    # None: the ambient default (_ops.parity_policy sets "fp32fwd", otherwise "bf16")
    encoder_precision = None

    @property
    def encoder_fp32(self) -> bool:
        return self.encoder_precision == "fp32"

    @encoder_fp32.setter
    def encoder_fp32(self, on: bool) -> None:
        self.encoder_precision = "fp32" if on else None

    def __init__(self, n_vocab, n_feats=None, encoder=None, decoder=None, cfm=None, data_statistics=None,
                 out_size=None, optimizer=None, scheduler=None, prior_loss=True, use_precomputed_durations=False,
                 out_channels=None, hidden_channels=None):
        super().__init__()
        self.n_vocab = n_vocab
        self.n_spks = 1
        self.out_size = out_size
        self.prior_loss = prior_loss
        self.use_precomputed_durations = use_precomputed_durations
        self.scheduler_config = scheduler
        if encoder is not None and decoder is not None and cfm is not None:  # :74-102
            self.n_feats = n_feats
            self.encoder = TextEncoder(encoder.encoder_type, encoder.encoder_params,
                                       encoder.duration_predictor_params, n_vocab)
            self.decoder = CFM(in_channels=2 * encoder.encoder_params.n_feats,
                               out_channel=encoder.encoder_params.n_feats, cfm_params=cfm, decoder_params=decoder)
        else:  # :104-176
            if out_channels is None or hidden_channels is None:
                raise ValueError("give either (encoder, decoder, cfm) configs or (out_channels, hidden_channels)")
            self.n_feats = out_channels
            enc = SimpleNamespace(
                encoder_type="transformer",
                encoder_params=SimpleNamespace(n_feats=out_channels, n_channels=hidden_channels, filter_channels=768,
                                               n_heads=2, n_layers=6, kernel_size=3, p_dropout=0.1, prenet=True),
                duration_predictor_params=SimpleNamespace(filter_channels_dp=256, kernel_size=3, p_dropout=0.1))
            self.encoder = TextEncoder(enc.encoder_type, enc.encoder_params, enc.duration_predictor_params, n_vocab)
            self.decoder = CFM(in_channels=2 * out_channels, out_channel=out_channels,
                               cfm_params=SimpleNamespace(solver="euler", sigma_min=1e-4),
                               decoder_params={"channels": (256, 256), "dropout": 0.05, "attention_head_dim": 64,
                                               "n_blocks": 1, "num_mid_blocks": 2, "num_heads": 4})
        if data_statistics is None:
            data_statistics = {"mel_mean": 0.0, "mel_std": 1.0}
        self.update_data_statistics(data_statistics)

    @torch.inference_mode()
    def synthesise(self, x, x_lengths, n_timesteps, temperature=1.0, length_scale=1.0, *, z=None):
        """matcha_tts.py:179-245 (reference fork).  ``z`` (keyword-only, [B, n_feats, y_max_length_])
        injects the ODE's initial noise for parity tests."""
        t0 = dt.datetime.now()
        mu_x, logw, x_mask = self.encoder(x, x_lengths)
        w_ceil = torch.ceil(torch.exp(logw) * x_mask) * length_scale
        y_lengths = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
        y_max_length = y_lengths.max()
        y_max_length_ = fix_len_compatibility(y_max_length)
        y_mask = sequence_mask(y_lengths, y_max_length_).unsqueeze(1).to(x_mask.dtype)
        attn_mask = x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)
        attn = generate_path(w_ceil.squeeze(1), attn_mask.squeeze(1)).unsqueeze(1)
        mu_y = torch.matmul(attn.squeeze(1).transpose(1, 2), mu_x.transpose(1, 2)).transpose(1, 2)
        decoder_outputs = self.decoder(mu_y, y_mask, n_timesteps, temperature, z=z)[:, :, :y_max_length]
        rtf = (dt.datetime.now() - t0).total_seconds() * 22050 / (decoder_outputs.shape[-1] * 256)
        return {"encoder_outputs": mu_y[:, :, :y_max_length], "decoder_outputs": decoder_outputs,
                "attn": attn[:, :, :y_max_length], "mel": denormalize(decoder_outputs, self.mel_mean, self.mel_std),
                "mel_lengths": y_lengths, "rtf": rtf}

    def log_prior(self, mu_x, y):
        """matcha_tts.py:277-282 in fp32: -1/2 sum y^2 + sum mu*y - 1/2 sum mu^2 - n/2 log(2 pi)."""
        with torch.autocast(device_type=mu_x.device.type, enabled=False):
            mu_x = mu_x.float()
            y = y.float()
            const = -0.5 * math.log(2 * math.pi) * self.n_feats
            factor = -0.5 * torch.ones(mu_x.shape, dtype=mu_x.dtype, device=mu_x.device)
            y_square = torch.matmul(factor.transpose(1, 2), y ** 2)
            y_mu_double = torch.matmul(2.0 * (factor * mu_x).transpose(1, 2), y)
            mu_square = torch.sum(factor * (mu_x ** 2), 1).unsqueeze(-1)
            return y_square - y_mu_double + mu_square + const

    def forward(self, x, x_lengths, y, y_lengths, out_size=None, cond=None, durations=None, *, t=None, z=None,
                segments=1):
        """Returns (dur_loss, prior_loss, diff_loss, attn) -- matcha_tts.py:247-325.  ``t``/``z``
        (keyword-only) inject the CFM randomness for parity tests.  ``segments`` = n > 1 (keyword-only, the
        Trainer's merged micro-batches): the batch is n equal micro-batches stacked along dim 0 and each loss
        is returned per micro-batch (a [n] tensor, every one normalised by its own micro-batch's lengths, as n
        separate forwards would) -- every other op of the model is per utterance."""
        # the text encoder runs on the same HIP GEMM/attention kernels as the decoder and follows the
        # caller's precision (bf16 MFMA operands inside a bf16 autocast region) unless encoder_precision says
        # otherwise: "bf16x3" / "fp32" take its activations' bf16 rounding -- what is left of the bf16 prior-loss
        # error and every alignment flip once the weights enter as split planes (tools/r3/precision_budget.py)
        # -- out of the forward
        # inside a Trainer step (the gradient deferral's side stream exists): the decoder's weight packs and
        # time path for this step's CFM time run on the side stream beside the text encoder (t drawn here
        # instead of in compute_loss; the same distribution)
        # t is drawn BEFORE the fork: the side stream's time embedding reads it, and the fork orders the side
        # stream after the main stream's work up to that point only (drawn after it, the read raced the draw)
        if x.is_cuda and _PREFETCH and t is None and O.side_fork_available():
            t = torch.rand([x.shape[0], 1, 1], device=x.device, dtype=torch.float32)
        side = O.side_fork() if (x.is_cuda and _PREFETCH) else None
        if side is not None:
            if t is None:
                t = torch.rand([x.shape[0], 1, 1], device=x.device, dtype=torch.float32)
            self.decoder.estimator.prefetch(t, side)
        enc_prec = self.encoder_precision or O.encoder_precision_default()
        if enc_prec == "fp32":
            enc_ctx = torch.autocast(device_type=x.device.type, enabled=False)
        elif enc_prec == "bf16x3":
            enc_ctx = O.precise_forward("bf16x3")
        elif enc_prec == "fp32fwd":
            enc_ctx = O.precise_forward("fp32")
        elif enc_prec == "bf16x6":
            enc_ctx = O.precise_forward("bf16x6")
        else:
            enc_ctx = _nullctx()
        with enc_ctx:
            mu_x, logw, x_mask = self.encoder(x, x_lengths)
        y_max_length = y.shape[-1]
        y_mask = O.sequence_mask_f32(y_lengths, y_max_length).unsqueeze(1)  # sequence_mask(...).to(x_mask), one launch
        runs = None
        if self.use_precomputed_durations:
            attn_mask = x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)
            attn = generate_path(durations.squeeze(1), attn_mask.squeeze(1))
            dur = torch.sum(attn, -1)
        else:
            # :276-288 fused on the GPU: lattice (log_prior) * attn_mask -> maximum_path -> sum(attn, -1),
            # with the attention mask taken from the lengths (never materialised)
            with torch.no_grad():
                attn, dur, col_row, row_start, lens = monotonic_align.prior_maximum_path(mu_x, y, x_lengths,
                                                                                          y_lengths)
            runs = (col_row, row_start, lens)
        # logw_ = log(1e-8 + dur) * x_mask ; duration_loss(logw, logw_, x_lengths)  (:287-288, model.py:117-135)
        # as one HIP launch each way
        if segments > 1:
            if x.shape[0] % segments:
                raise ValueError(f"segments={segments} does not divide the batch {x.shape[0]}")
            bs = x.shape[0] // segments
            dur_loss = torch.stack([O.duration_loss_fused(logw[i * bs:(i + 1) * bs], dur[i * bs:(i + 1) * bs],
                                                          x_lengths[i * bs:(i + 1) * bs]) for i in range(segments)])
        else:
            dur_loss = O.duration_loss_fused(logw, dur, x_lengths)
        if out_size is not None:  # :290-312 (host-side random crop, as the reference)
            max_offset = (y_lengths - out_size).clamp(0)
            offset_ranges = list(zip([0] * max_offset.shape[0], max_offset.cpu().numpy()))
            out_offset = torch.LongTensor([random.choice(range(s, e)) if e > s else 0
                                           for s, e in offset_ranges]).to(y_lengths)
            attn_cut = torch.zeros(attn.shape[0], attn.shape[1], out_size, dtype=attn.dtype, device=attn.device)
            y_cut = torch.zeros(y.shape[0], self.n_feats, out_size, dtype=y.dtype, device=y.device)
            y_cut_lengths = []
            for i, (y_, off) in enumerate(zip(y, out_offset)):
                L = out_size + (y_lengths[i] - out_size).clamp(None, 0)
                y_cut_lengths.append(L)
                y_cut[i, :, :L] = y_[:, off:off + L]
                attn_cut[i, :, :L] = attn[i, :, off:off + L]
            y_cut_lengths = torch.LongTensor(y_cut_lengths)
            y_mask = sequence_mask(y_cut_lengths).unsqueeze(1).to(y_mask)
            attn, y = attn_cut, y_cut
            runs = None
        if runs is not None:  # attn^T @ mu_x on the one-hot attn == a gather (bitwise), segment-sum backward
            mu_y = monotonic_align.expand_rows(mu_x, *runs)
        else:
            mu_y = torch.matmul(attn.squeeze(1).transpose(1, 2), mu_x.transpose(1, 2)).transpose(1, 2)
        # CFM loss (:317) and prior loss (:319-323) in one fused HIP pass (components/flow_matching.py)
        diff_loss, prior_loss, _ = self.decoder.compute_loss_and_prior(y, y_mask, mu_y,
                                                                       mu_y if self.prior_loss else None, t=t, z=z,
                                                                       segments=segments)
        if not self.prior_loss:
            prior_loss = 0
        return dur_loss, prior_loss, diff_loss, attn
