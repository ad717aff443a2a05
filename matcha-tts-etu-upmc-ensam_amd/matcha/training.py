"""Train-step driver: the semantics of the reference's Lightning loop (train.py:81-102,
baselightningmodule.py:115-162) on one process per GPU.

  - fp32 master weights, AdamW(1e-4, (0.9, 0.999), wd 1e-6) + per-epoch cosine (configure_optimizers)
  - gradient clipping by global norm 1.0 (gradient_clip_val=1.0)
  - gradient accumulation (accumulate_grad_batches; the reference uses 2 x 16 = 32 per step)
  - data parallel over RCCL: torch DDP buckets the gradients (bucket_mb) and all-reduces each bucket
    on its comm stream as soon as backward has produced it, i.e. overlapped with the rest of
    backward; non-final accumulation micro-batches skip the all-reduce (no_sync)
  - the 4 logged losses of a step are reduced in ONE all-reduce (the reference issues one
    sync_dist all-reduce per self.log call)

Synthetic LJSpeech-shaped batches: token ids ~ U{1..149}, lengths ~ U[0.7 max, max]
with element 0 = max, mels ~ N(0, 1) zeroed past the length.
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass

import torch
import torch.distributed as dist

from matcha.models.matcha_tts import MatchaTTS


def synthetic_batch(B: int, Tx: int, Ty: int, n_feats: int = 80, seed: int = 0, device="cuda",
                    n_vocab: int = 150) -> dict:
    g = torch.Generator().manual_seed(seed)
    x_lengths = (Tx * (0.7 + 0.3 * torch.rand(B, generator=g))).long().clamp(1, Tx)
    y_lengths = (Ty * (0.7 + 0.3 * torch.rand(B, generator=g))).long().clamp(1, Ty)
    x_lengths[0], y_lengths[0] = Tx, Ty
    y_lengths = torch.maximum(y_lengths, x_lengths)
    x = torch.randint(1, n_vocab, (B, Tx), generator=g)
    y = torch.randn(B, n_feats, Ty, generator=g)
    pos_x = torch.arange(Tx)[None, :]
    pos_y = torch.arange(Ty)[None, None, :]
    x = x * (pos_x < x_lengths[:, None])
    y = y * (pos_y < y_lengths[:, None, None])
    return {k: v.to(device) for k, v in dict(x=x, x_lengths=x_lengths, y=y, y_lengths=y_lengths).items()}


@dataclass
class TrainConfig:
    accumulate_grad_batches: int = 1
    gradient_clip_val: float = 1.0
    bucket_mb: float = 25.0
    precision: str = "32-true"  # "32-true" (reference) or "bf16-mixed"


class Trainer:
    def __init__(self, model: MatchaTTS, cfg: TrainConfig = TrainConfig()):
        self.cfg = cfg
        self.model = model
        self.ddp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        if self.ddp:
            dev = next(model.parameters()).device
            self.wrapped = torch.nn.parallel.DistributedDataParallel(
                model, device_ids=[dev.index], bucket_cap_mb=cfg.bucket_mb, gradient_as_bucket_view=True,
                broadcast_buffers=False)
        else:
            self.wrapped = model
        opt = model.configure_optimizers()
        self.optimizer = opt["optimizer"]
        self.scheduler = opt["lr_scheduler"]["scheduler"]
        self.global_step = 0
        self.last_losses = None

    def _autocast(self):
        if self.cfg.precision == "bf16-mixed":
            return torch.autocast(device_type="cuda", dtype=torch.bfloat16)
        return contextlib.nullcontext()

    def step(self, batches: list[dict]) -> torch.Tensor:
        """One optimizer step over len(batches) == accumulate_grad_batches micro-batches.
        Returns the device tensor [dur, prior, diff, total] (mean over micro-batches and ranks);
        nothing here synchronises with the host."""
        assert len(batches) == self.cfg.accumulate_grad_batches
        n = len(batches)
        logged = None
        for i, batch in enumerate(batches):
            sync = i == n - 1
            ctx = self.wrapped.no_sync() if (self.ddp and not sync) else contextlib.nullcontext()
            with ctx:
                with self._autocast():
                    dur, prior, diff, _ = self.wrapped(x=batch["x"], x_lengths=batch["x_lengths"],
                                                       y=batch["y"], y_lengths=batch["y_lengths"])
                    total = dur + prior + diff
                (total / n).backward()
            vals = torch.stack([dur.detach(), torch.as_tensor(prior).detach(), diff.detach(), total.detach()]).float()
            logged = vals if logged is None else logged + vals
        logged = logged / n
        if self.ddp:  # the step's logged scalars in one collective (sync_dist=True)
            dist.all_reduce(logged)
            logged = logged / dist.get_world_size()
        if self.cfg.gradient_clip_val:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.cfg.gradient_clip_val, foreach=True)
        self.optimizer.step()
        self.optimizer.zero_grad(set_to_none=True)
        self.global_step += 1
        self.last_losses = logged
        return logged

    def on_epoch_end(self):
        self.scheduler.step()
