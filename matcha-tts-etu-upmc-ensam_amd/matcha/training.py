"""Train-step driver: the semantics of the reference's Lightning loop (train.py:81-102,
baselightningmodule.py:115-162) on one process per GPU.

  - fp32 master weights, AdamW(1e-4, (0.9, 0.999), wd 1e-6) + per-epoch cosine (configure_optimizers)
  - gradient clipping by global norm 1.0 (gradient_clip_val=1.0)
  - gradient accumulation (accumulate_grad_batches; the reference uses 2 x 16 = 32 per step)
  - the step's 4 logged losses reduced in ONE collective (the reference issues one sync_dist
    all-reduce per self.log call)

Two execution modes:
  graph=True (default on GPU): the whole step is captured once into a HIP graph and replayed -- about
    a thousand kernel launches per step become one graph launch.  Gradients are NOT pre-allocated:
    param.grad is None when backward starts, so autograd hands each parameter its freshly computed
    gradient tensor (no per-parameter accumulate kernel).  N=1: clip + AdamW read those tensors inside
    the same graph.  N>1: one batched copy packs them into a flat fp32 buffer, data parallelism is a
    single RCCL all-reduce of that buffer over xGMI, and a second graph runs clip + AdamW on views of
    it.  Dropout masks
    (torch's and the HIP epilogues') are drawn from device-side RNG state, so every replay draws new
    masks.  Inputs are copied into static buffers before each replay.
  graph=False (eager): torch DDP over RCCL (bucketed all-reduce overlapped with backward, no_sync
    for non-final accumulation micro-batches).

Synthetic LJSpeech-shaped batches: token ids ~ U{1..149}, lengths ~ U[0.7 max, max]
with element 0 = max, mels ~ N(0, 1) zeroed past the length.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from matcha import _native as N
from matcha.models.components import _ops as OPS
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


class _AdamWChunk(ctypes.Structure):  # include/mtts_decoder.h mtts_adamw_chunk
    _fields_ = [("grad", ctypes.c_void_p), ("offset", ctypes.c_int64), ("n", ctypes.c_int32), ("pad_", ctypes.c_int32)]


class _FlatClipAdamW:
    """clip_grad_norm_(max_norm) + AdamW(lr, (0.9, 0.999), eps 1e-8, wd 1e-6) -- the reference step's
    optimizer (baselightningmodule.py:59-65, train.py gradient_clip_val) -- as mtts_clip_adamw over a
    flat parameter array.  lr is a float64 device scalar (the cosine schedule writes it); the step count lives
    on the device; the gradient table is rebuilt whenever the gradient tensors change (eager calls)
    and frozen by bind_grads() for graph capture."""

    CHUNK = 32768

    def __init__(self, params, lr: torch.Tensor, max_norm: float, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-6):
        if lr.dtype != torch.float64:
            raise TypeError("lr must be a float64 device scalar (torch derives AdamW's scalars in double)")
        self.params = list(params)
        dev = self.params[0].device
        offs, off = [], 0
        for p in self.params:
            offs.append(off)
            off += (p.numel() + 3) // 4 * 4
        self.flat = torch.zeros(off, device=dev, dtype=torch.float32)
        with torch.no_grad():
            for p, o in zip(self.params, offs):
                self.flat[o:o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = self.flat[o:o + p.numel()].view_as(p)
        self.offsets = offs
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.step_t = torch.zeros(1, device=dev, dtype=torch.float32)
        self.lr, self.max_norm = lr, float(max_norm or 0.0)
        self.betas, self.eps, self.wd = betas, eps, weight_decay
        self._table = None
        self._key = None
        self._ws = None
        self.state = {}  # (torch.optim API surface used by callers)

    def _build(self):
        key = tuple((p.grad.data_ptr() if p.grad is not None else 0) for p in self.params)
        if key == self._key:
            return
        rows = []
        for p, o in zip(self.params, self.offsets):
            g = p.grad
            if g is None:
                continue
            if g.dtype != torch.float32 or not g.is_contiguous():
                raise RuntimeError("fused AdamW expects contiguous fp32 gradients")
            n = g.numel()
            for s in range(0, n, self.CHUNK):
                rows.append((g.data_ptr() + 4 * s, o + s, min(self.CHUNK, n - s)))
        arr = (_AdamWChunk * max(len(rows), 1))()
        for i, (gp, o, n) in enumerate(rows):
            arr[i].grad, arr[i].offset, arr[i].n = gp, o, n
        host = torch.frombuffer(bytearray(arr), dtype=torch.uint8)
        self._table = host.to(self.flat.device)
        self._n = len(rows)
        nws = int(N.lib().mtts_clip_adamw_workspace_size(self._n))
        self._ws = torch.empty(max(nws, 4), dtype=torch.uint8, device=self.flat.device)
        self._key = key

    def bind_grads(self):
        self._key = None
        self._build()

    def step(self):
        if torch.cuda.is_current_stream_capturing():
            if self._table is None:
                raise RuntimeError("bind_grads() before capturing the optimizer step")
        else:
            self._build()
        b1, b2 = self.betas
        N.check(N.lib().mtts_clip_adamw(N.ptr(self._table), self._n, N.ptr(self.flat), N.ptr(self.exp_avg),
                                        N.ptr(self.exp_avg_sq), N.ptr(self.lr), N.ptr(self.step_t), self.max_norm,
                                        b1, b2, self.eps, self.wd, N.ptr(self._ws), self._ws.numel(),
                                        torch.cuda.current_stream(self.flat.device).cuda_stream), "mtts_clip_adamw")

    def state_snapshot(self):
        return [t.clone() for t in (self.exp_avg, self.exp_avg_sq, self.step_t)]

    def state_restore(self, snap):
        for t, s_ in zip((self.exp_avg, self.exp_avg_sq, self.step_t), snap):
            t.copy_(s_)

    def zero_grad(self, set_to_none: bool = True):
        for p in self.params:
            p.grad = None


N.register("mtts_clip_adamw_workspace_size", ctypes.c_size_t, [ctypes.c_int32])
N.register("mtts_clip_adamw", ctypes.c_int,
           [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_float, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p])


@dataclass
class TrainConfig:
    accumulate_grad_batches: int = 1
    gradient_clip_val: float = 1.0
    bucket_mb: float = 25.0
    precision: str = "32-true"  # "32-true" (reference) or "bf16-mixed"
    graph: bool = False
    lr: float = 1e-4
    eta_min: float = 1e-6
    t_max_epochs: int = 1000


class Trainer:
    # opt-in: measured in-step on MI355X the graph step got 0.25 ms SLOWER with weight gradients on a
    # side stream (11.25 vs 11.01 ms): the ~100 cross-stream edges cost more than the overlap returns
    side_stream_wgrad = os.environ.get("MTTS_SIDE_WGRAD", "0") == "1"
    defer_grad_sums = os.environ.get("MTTS_DEFER_GRAD_SUMS", "1") != "0"

    def __init__(self, model: MatchaTTS, cfg: TrainConfig = TrainConfig()):
        self.cfg = cfg
        self.model = model
        self.world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
        self.dev = next(model.parameters()).device
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.global_step = 0
        self.epoch = 0
        self.last_losses = None
        if cfg.graph:
            if self.world > 1:  # identical initial weights on every rank (what DDP's broadcast does)
                for p in model.state_dict().values():
                    dist.broadcast(p, 0)
            self.flat = None  # N>1: packed gradients for the all-reduce (sized at capture)
            for p in self.params:
                p.grad = None
            self.lr = torch.tensor(cfg.lr, device=self.dev, dtype=torch.float64)  # torch keeps lr a double
            # clip + AdamW as two HIP launches (csrc/optim.hip) over one flat fp32 parameter array:
            # the parameters become views into it (names / state_dict unchanged), each region
            # 16-byte aligned; the moments are flat arrays of the same layout
            self.optimizer = _FlatClipAdamW(self.params, self.lr, cfg.gradient_clip_val)
            self.scheduler = None
            self._g_fb = self._g_opt = None
            self._static = None
            self.wrapped = model
        else:
            if self.world > 1:
                self.wrapped = torch.nn.parallel.DistributedDataParallel(
                    model, device_ids=[self.dev.index] if self.dev.type == "cuda" else None,
                    bucket_cap_mb=cfg.bucket_mb, gradient_as_bucket_view=True, broadcast_buffers=False)
            else:
                self.wrapped = model
            opt = model.configure_optimizers()
            self.optimizer = opt["optimizer"]
            self.scheduler = opt["lr_scheduler"]["scheduler"]

    # ------------------------------------------------------------------------------------ common
    def _autocast(self):
        if self.cfg.precision == "bf16-mixed" and self.dev.type == "cuda":
            return torch.autocast(device_type="cuda", dtype=torch.bfloat16)
        return contextlib.nullcontext()

    def _fwd_bwd(self, batches, sync_ctx=None):
        n = len(batches)
        # weight gradients on a side stream, overlapping the dgrad chain (components/_ops.py
        # side_stream_wgrad): safe when autograd steals every fresh gradient (graph step, one
        # micro-batch, gradients set to None first); joined before this returns
        fresh = n == 1 and self.dev.type == "cuda" and all(p.grad is None for p in self.params)
        side = self.cfg.graph and fresh and self.side_stream_wgrad
        # the parameter-gradient partial sums of the whole backward in one batched launch
        # (components/_ops.py deferred_grad_sums): also needs fresh gradients, and no DDP hook
        # reading them during the backward
        defer = fresh and self.defer_grad_sums and not side and (self.cfg.graph or self.world == 1)
        with OPS.deferred_grad_sums(defer), OPS.side_stream_wgrad(side):
            return self._fwd_bwd_body(batches, sync_ctx)

    def _fwd_bwd_body(self, batches, sync_ctx=None):
        n = len(batches)
        logged = None
        for i, batch in enumerate(batches):
            ctx = sync_ctx(i) if sync_ctx else contextlib.nullcontext()
            with ctx:
                with self._autocast():
                    dur, prior, diff, _ = self.wrapped(x=batch["x"], x_lengths=batch["x_lengths"],
                                                       y=batch["y"], y_lengths=batch["y_lengths"])
                    total = dur + prior + diff
                (total / n).backward()
            vals = torch.stack([dur.detach(), torch.as_tensor(prior).detach(), diff.detach(), total.detach()]).float()
            logged = vals if logged is None else logged + vals
        return logged / n

    def _clip_and_update(self):
        if isinstance(self.optimizer, _FlatClipAdamW):  # graph mode: clipping is inside the fused step
            self.optimizer.step()
            return
        if self.cfg.gradient_clip_val:
            torch.nn.utils.clip_grad_norm_(self.params, self.cfg.gradient_clip_val, foreach=True)
        self.optimizer.step()

    # ------------------------------------------------------------------------------------ eager
    def _eager_step(self, batches):
        n = len(batches)
        ddp = self.world > 1

        def sync_ctx(i):
            return self.wrapped.no_sync() if (ddp and i < n - 1) else contextlib.nullcontext()

        logged = self._fwd_bwd(batches, sync_ctx)
        if ddp:  # the step's logged scalars in one collective (sync_dist=True)
            dist.all_reduce(logged)
            logged = logged / self.world
        self._clip_and_update()
        self.optimizer.zero_grad(set_to_none=True)
        return logged

    # ------------------------------------------------------------------------------------ graph
    def _graph_capture(self, batches):
        self._static = [{k: v.clone() for k, v in b.items()} for b in batches]
        # warm-up (allocator pools, lazy library loads, optimizer state) must not leave updates behind
        saved = [p.detach().clone() for p in self.params]
        saved_state = self.optimizer.state_snapshot()
        side = torch.cuda.Stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                for p in self.params:
                    p.grad = None
                self._fwd_bwd(self._static)
                self._clip_and_update()
        torch.cuda.current_stream(self.dev).wait_stream(side)
        gparams = [p for p in self.params if p.grad is not None]  # parameters the step differentiates
        with torch.no_grad():
            for p, s_ in zip(self.params, saved):
                p.copy_(s_)
            self.optimizer.state_restore(saved_state)  # moments / step back to their pre-warm-up values

        if self.world > 1:
            self.flat = torch.zeros(sum(p.numel() for p in gparams), device=self.dev, dtype=torch.float32)
        self._g_fb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_fb):
            for p in self.params:
                p.grad = None  # autograd hands over each fresh gradient: no accumulate kernels
            self._logged = self._fwd_bwd(self._static)
            if self.world > 1:
                torch.cat([p.grad.reshape(-1) for p in gparams], out=self.flat)
        self._fb_grads = [p.grad for p in gparams]  # graph-pool outputs, kept alive with the graph
        if self.world > 1:
            off = 0
            for p in gparams:  # the optimizer graph reads the all-reduced flat buffer
                p.grad = self.flat[off:off + p.numel()].view_as(p)
                off += p.numel()
        # the optimizer graph: its gradient table points at the (fixed) graph-pool gradients
        self.optimizer.bind_grads()
        self._g_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_opt, pool=self._g_fb.pool()):
            self._clip_and_update()

    def _graph_step(self, batches):
        if self._g_fb is None or len(batches) != len(self._static) or any(
                b[k].shape != s[k].shape for b, s in zip(batches, self._static) for k in s):
            self._graph_capture(batches)
        for b, s in zip(batches, self._static):
            for k, v in s.items():
                if b[k] is not v:
                    v.copy_(b[k], non_blocking=True)
        self._g_fb.replay()
        logged = self._logged
        if self.world > 1:
            dist.all_reduce(self.flat)  # one RCCL all-reduce of every gradient
            self.flat.div_(self.world)
            logged = logged.clone()
            dist.all_reduce(logged)
            logged = logged / self.world
        self._g_opt.replay()
        return logged

    # ------------------------------------------------------------------------------------ api
    def step(self, batches: list[dict]) -> torch.Tensor:
        """One optimizer step over len(batches) == accumulate_grad_batches micro-batches.  Returns the
        device tensor [dur, prior, diff, total] (mean over micro-batches and ranks); nothing here
        synchronises with the host."""
        assert len(batches) == self.cfg.accumulate_grad_batches
        logged = self._graph_step(batches) if self.cfg.graph else self._eager_step(batches)
        self.global_step += 1
        self.last_losses = logged
        return logged

    def on_epoch_end(self):
        """CosineAnnealingLR(T_max=1000 epochs, eta_min=1e-6) stepped per epoch."""
        self.epoch += 1
        if self.scheduler is not None:
            self.scheduler.step()
        else:
            c = self.cfg
            lr = c.eta_min + (c.lr - c.eta_min) * (1 + math.cos(math.pi * self.epoch / c.t_max_epochs)) / 2
            self.lr.fill_(lr)
