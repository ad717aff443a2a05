"""Train-step driver: the semantics of the reference's Lightning loop (train.py:81-102,
baselightningmodule.py:115-162) on one process per GPU.

  - fp32 master weights, AdamW(1e-4, (0.9, 0.999), eps 1e-8, wd 1e-6) + per-epoch cosine
    (configure_optimizers)
  - gradient clipping by global norm 1.0 (gradient_clip_val=1.0)
  - gradient accumulation (accumulate_grad_batches; the reference uses 2 x 16 = 32 per step)
  - the step's 4 logged losses reduced in ONE collective (the reference issues one sync_dist
    all-reduce per self.log call)

Two execution modes:
  graph=True (default on GPU): the whole step is captured once per input shape into a HIP graph and
    replayed (shape-keyed LRU cache, TrainConfig.graph_cache) -- about a thousand kernel launches per
    step become one graph launch.  Gradients are NOT pre-allocated: param.grad is None when backward
    starts, so autograd hands each parameter its freshly computed gradient tensor (no per-parameter
    accumulate kernel).  N=1: clip + AdamW (csrc/optim.hip, over one flat parameter array) run in a
    second graph on those tensors.  N>1 (matcha/dp.py): post-accumulate-grad hooks pack the gradients
    bucket by bucket into a flat fp32 buffer and fork each bucket's RCCL all-reduce (libmtts_hip's own
    communicator, capturable) onto a side stream while backward continues; the join, clip and AdamW on
    views of the reduced buffer are in the SAME graph.  With torch.distributed as the transport (gloo,
    the shared-GPU rehearsal) the graph only packs, the host reduces the flat buffer, and a second
    graph steps.  Dropout masks (torch's and the HIP epilogues') come from device-side RNG state, so
    every replay draws new masks.  Inputs are copied into static buffers before each replay.
  graph=False (eager): torch DDP over RCCL (bucketed all-reduce overlapped with backward, no_sync for
    non-final accumulation micro-batches), or the same bucket reducer (dp="buckets").

N>1 graph step: every replay issues the same collective sequence (the buckets of one fixed layout -- rank
0's recorded backward order, broadcast once -- in bucket order), whatever shape a rank's batch has; a
capture's warm-up passes never communicate (the reducer packs only), and the communicator's connections
are set up once by an eager all-reduce per bucket on every rank when the reducer is built.  By default
(TrainConfig.agree_shapes=True) every rank pads to the MAX padded Tx / Ty over ranks -- one host-side gloo
all-reduce per step, no GPU sync -- so all ranks capture and replay the same graph together; the extra padding
changes the padded-length dependent parts of the arithmetic (GroupNorm statistics, conv bias leaking into padded
frames).  agree_shapes=False lets each rank pad to its own length, as the reference's DDP would, and capture new
shapes on its own (tested over gloo; not yet run with the in-graph RCCL transport on a multi-GPU box).

Synthetic LJSpeech-shaped batches: token ids ~ U{1..149}, lengths ~ U[0.7 max, max]
with element 0 = max, mels ~ N(0, 1) zeroed past the length.  A batch dict may carry "t" [B, 1, 1] and
"z" [B, n_feats, Ty]: the CFM randomness injected for parity tests (MatchaTTS.forward's keywords).
"""
from __future__ import annotations

import collections
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
        # gradients are SUMS over grad_scale^-1 data-parallel ranks (RcclComm: ncclSum); the mean is taken here
        self.grad_scale = 1.0
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
        N.check(N.lib().mtts_clip_adamw_scaled(N.ptr(self._table), self._n, N.ptr(self.flat), N.ptr(self.exp_avg),
                                               N.ptr(self.exp_avg_sq), N.ptr(self.lr), N.ptr(self.step_t),
                                               self.max_norm, b1, b2, self.eps, self.wd, self.grad_scale,
                                               N.ptr(self._ws), self._ws.numel(),
                                               torch.cuda.current_stream(self.flat.device).cuda_stream),
                "mtts_clip_adamw_scaled")

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
N.register("mtts_clip_adamw_scaled", ctypes.c_int,
           [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_float, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
            ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p])


@dataclass
class TrainConfig:
    accumulate_grad_batches: int = 1
    gradient_clip_val: float = 1.0
    bucket_mb: float = 25.0  # DDP buckets (eager) and the graph step's all-reduce buckets
    # graph step: one bucket boundary at the decoder / encoder seam of the backward (the decoder's gradients are
    # issued together where the N=1 step side-flushes them), buckets up to seam_bucket_mb inside each part.
    # Round 4, forced-DP step on one GPU: 25 MB buckets flushed the queued weight gradients mid-decoder-backward
    # (+0.39 ms over the plain step); False: plain bucket_mb buckets
    bucket_seams: bool = True
    seam_bucket_mb: float = 64.0
    # "32-true" (reference), "bf16-mixed" (autocast), or "bf16-parity": bf16-mixed with split bf16 weight
    # planes (every forward GEMM but the decoder FF's GELU up-projection) and the text encoder's forward on the
    # exact-fp32 MFMA -- alignment exact, losses within 1e-4 of 32-true
    # (tests/test_headline_gpu.py; _ops.parity_policy)
    precision: str = "32-true"
    graph: bool = False
    lr: float = 1e-4
    eta_min: float = 1e-6
    t_max_epochs: int = 1000
    # captured steps kept per input-shape key (LRU); collate(x_quantum=16, y_quantum=64) on bucketed batches
    # keeps real data to ~20 padded shapes (tests/test_data_path.py) -- size the cache to cover them.  Each
    # cached graph keeps its own memory pool holding the whole step's activations and gradients (~2-3 GB at
    # B=32 x 600 frames bf16-mixed, ~6 GB at B=8 x 4096): 20 shapes fit the MI355X's 288 GB many times
    graph_cache: int = 4
    dp: str = "auto"  # N>1 exchange: "ddp" (eager only), "buckets" (GradBucketReducer), "auto"
    comm: str = "auto"  # bucket reducer transport: "rccl" (capturable, libmtts_hip), "torch", "auto"
    # N>1 graph step: pad every rank's batch to the MAX padded shape over ranks (see the module docstring), so
    # every rank captures and replays the same graph and issues the same in-graph RCCL collectives.  ON by default
    # (ADVICE r4): rank-local captures beside peers that replay in-graph RCCL all-reduces have never run on a
    # multi-GPU box; False keeps each rank's own padding (as DDP in the reference's setup) -- exercised over gloo
    # by tests/test_dp_multirank_gpu.py
    agree_shapes: bool = True
    # run the data-parallel exchange even at world size 1 (a world-size-1 process group must exist): the
    # bucketed RCCL path's cost on one GPU (bench.py extra_configs.dp_forced_n1); MTTS_FORCE_DP=1 does the same
    force_dp: bool = False
    # accumulate_grad_batches > 1 with micro-batches of one padded shape: ONE forward / backward of the stacked
    # micro-batches, each loss normalised per micro-batch (MatchaTTS.forward(segments=n)) -- the gradient of
    # (1/n) sum_i L_i that accumulation computes; every op but the losses is per utterance (GroupNorm / LayerNorm
    # statistics per utterance and padded length), so only the weight-gradient reductions' rounding differs.
    # Micro-batches of different padded shapes take the stashed fresh-gradient path (_fwd_bwd_stash)
    merge_micro_batches: bool = True


class Trainer:
    # opt-in: measured in-step on MI355X the graph step got SLOWER with weight gradients on a side
    # stream (round 1: 11.25 vs 11.01 ms; round 2: 9.43 vs 8.57 ms): the ~100 cross-stream edges cost
    # more than the overlap returns
    side_stream_wgrad = os.environ.get("MTTS_SIDE_WGRAD", "0") == "1"
    defer_grad_sums = os.environ.get("MTTS_DEFER_GRAD_SUMS", "1") != "0"
    # MTTS_FORCE_DP=1: run the data-parallel exchange even at world size 1 (rehearses the bucketed
    # RCCL path on a one-GPU box; the all-reduce of one rank is a copy)
    force_dp = os.environ.get("MTTS_FORCE_DP", "0") == "1"

    def __init__(self, model: MatchaTTS, cfg: TrainConfig = TrainConfig()):
        self.cfg = cfg
        self.model = model
        self.world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
        self.dev = next(model.parameters()).device
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.global_step = 0
        self.epoch = 0
        self.last_losses = None
        self.dp = self.world > 1 or ((self.force_dp or cfg.force_dp) and dist.is_available() and dist.is_initialized())
        mode = cfg.dp if cfg.dp != "auto" else ("buckets" if cfg.graph else "ddp")
        if cfg.graph and mode == "ddp":
            raise ValueError("the graph step exchanges gradients with the bucket reducer (dp='buckets')")
        self.dp_mode = mode if self.dp else None
        self.reducer = None
        self._recorder = None
        self._arm = None  # (overlap,) while the reducer is to be armed in the next backward
        self._graphs = collections.OrderedDict()
        # bench.py's N>1 path (matcha/watchdog.py): a host watchdog told of every step / graph key / bucket issue,
        # and device progress markers captured into the step (one after each bucket's all-reduce, one at its end)
        self.watchdog = None
        self.progress = None
        # a gloo group for the host-side agreements (padded shapes, bucket layout): never syncs the GPU
        self._host_group = None
        if self.dp and self.world > 1:
            if dist.get_backend() == "gloo":
                self._host_group = dist.group.WORLD
            else:
                from matcha.dp import stdout_to_stderr

                with stdout_to_stderr():  # gloo's connect message stays off the bench's JSON stdout
                    self._host_group = dist.new_group(backend="gloo")
        if self.dp and self.world > 1:  # identical initial weights on every rank (what DDP's broadcast does)
            for p in model.state_dict().values():
                dist.broadcast(p, 0)
        if cfg.graph:
            for p in self.params:
                p.grad = None
            self.lr = torch.tensor(cfg.lr, device=self.dev, dtype=torch.float64)  # torch keeps lr a double
            # clip + AdamW as two HIP launches (csrc/optim.hip) over one flat fp32 parameter array:
            # the parameters become views into it (names / state_dict unchanged), each region
            # 16-byte aligned; the moments are flat arrays of the same layout
            self.optimizer = _FlatClipAdamW(self.params, self.lr, cfg.gradient_clip_val)
            self.scheduler = None
            self.wrapped = model
        else:
            if self.dp_mode == "ddp":
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
        if self.cfg.precision in ("bf16-mixed", "bf16-parity") and self.dev.type == "cuda":
            st = contextlib.ExitStack()
            st.enter_context(torch.autocast(device_type="cuda", dtype=torch.bfloat16))
            if self.cfg.precision == "bf16-parity":
                st.enter_context(OPS.parity_policy())
            return st
        return contextlib.nullcontext()

    def _fwd_bwd(self, batches, sync_ctx=None):
        n = len(batches)
        if n > 1 and self._merge_ok(batches):
            batches = [self._merge(batches)]
            n = 1
        elif n > 1 and self._stash_ok():
            return self._fwd_bwd_stash(batches)
        # weight gradients on a side stream, overlapping the dgrad chain (components/_ops.py
        # side_stream_wgrad): safe when autograd steals every fresh gradient (graph step, one
        # micro-batch, gradients set to None first); joined before this returns
        fresh = n == 1 and self.dev.type == "cuda" and all(p.grad is None for p in self.params)
        # (never with the DP reducer: it packs gradients on the main stream while the side stream may
        # still be writing them)
        side = self.cfg.graph and fresh and self.side_stream_wgrad and not self.dp
        # the parameter-gradient partial sums of the whole backward in one batched launch
        # (components/_ops.py deferred_grad_sums): also needs fresh gradients, and no DDP hook
        # reading them during the backward (the bucket reducer flushes the queue per bucket)
        defer = fresh and self.defer_grad_sums and not side and (self.cfg.graph or self.dp_mode != "ddp")
        # several micro-batches (accumulate_grad_batches): the FIRST one's gradients are fresh too -- its
        # backward runs deferred (batched weight gradients, flushed when it ends, before the next micro-batch
        # accumulates into them); the later ones accumulate and run per layer
        self._defer_first = (n > 1 and self.dev.type == "cuda" and self.defer_grad_sums
                             and all(p.grad is None for p in self.params)
                             and (self.cfg.graph or self.dp_mode != "ddp"))
        with OPS.deferred_grad_sums(defer), OPS.side_stream_wgrad(side):
            return self._fwd_bwd_body(batches, sync_ctx)

    def _merge_ok(self, batches) -> bool:
        """TrainConfig.merge_micro_batches and every micro-batch the same padded shapes (CUDA MatchaTTS)."""
        if not self.cfg.merge_micro_batches or self.dev.type != "cuda" or not isinstance(self.model, MatchaTTS):
            return False
        keys = set(batches[0])
        return all(set(b) == keys and all(b[k].shape == batches[0][k].shape and b[k].dtype == batches[0][k].dtype
                                          for k in keys) for b in batches[1:]) and "_segments" not in keys

    @staticmethod
    def _merge(batches):
        out = {k: torch.cat([b[k] for b in batches], 0) for k in batches[0]}
        out["_segments"] = len(batches)
        return out

    def _stash_ok(self) -> bool:
        """accumulate_grad_batches > 1 without data parallelism: every micro-batch can take the fresh-gradient
        path (batched, deferred weight gradients and sums, side-stream seam flushes) -- its gradients are
        stashed and summed at the end instead of accumulated per layer.  The DP reducer packs the last
        micro-batch's gradients as backward produces them, so it keeps the accumulating path."""
        return (self.dev.type == "cuda" and not self.dp and self.defer_grad_sums
                and all(p.grad is None for p in self.params))

    def _fwd_bwd_stash(self, batches):
        """Micro-batch i: forward + (total / n).backward() on fresh gradients under the gradient deferral (the
        N=1 step's fast path), its gradients stashed; the end sums them with multi-tensor adds in micro-batch
        order, ((g_1 + g_2) + g_3) ..., the fp32 adds autograd's AccumulateGrad does -- so the result equals
        the accumulating path's (tests/test_training_gpu.py::test_accumulate_grad_batches_2_vs_torch)."""
        n = len(batches)
        self._defer_first = False
        logged = None
        stash = []
        for i, batch in enumerate(batches):
            with OPS.deferred_grad_sums(True):
                vals = self._fwd_bwd_body([batch], div=n)
            logged = vals if logged is None else logged + vals
            stash.append([p.grad for p in self.params])
            for p in self.params:
                p.grad = None
        acc = list(stash[0])
        for g in stash[1:]:
            a_, b_ = [], []
            for k, gk in enumerate(g):
                if gk is None:
                    continue
                if acc[k] is None:
                    acc[k] = gk
                else:
                    a_.append(acc[k])
                    b_.append(gk)
            if a_:
                torch._foreach_add_(a_, b_)  # in place into micro-batch 1's (fresh, unaliased) gradients
        for p, gk in zip(self.params, acc):
            p.grad = gk
        return logged / n

    def _fwd_bwd_body(self, batches, sync_ctx=None, div=None):
        n = len(batches)
        logged = None
        for i, batch in enumerate(batches):
            ctx = sync_ctx(i) if sync_ctx else contextlib.nullcontext()
            first = OPS.deferred_grad_sums(True) if (i == 0 and getattr(self, "_defer_first", False)) \
                else contextlib.nullcontext()
            with ctx, first:
                inject = {k: batch[k] for k in ("t", "z") if k in batch}  # parity tests' CFM randomness
                seg = batch.get("_segments", 1)
                if seg > 1:  # merged micro-batches: per-micro-batch losses ([seg] tensors)
                    inject["segments"] = seg
                with self._autocast():
                    dur, prior, diff, _ = self.wrapped(x=batch["x"], x_lengths=batch["x_lengths"],
                                                       y=batch["y"], y_lengths=batch["y_lengths"], **inject)
                # total = dur + prior + diff and the logged [dur, prior, diff, total] in one launch (device
                # tensors; the CPU data-parallel tests drive this loop with a CPU stand-in model)
                if seg > 1:  # the mean over micro-batches of each one's total / logged vector
                    parts = [OPS.loss_sum(dur[j], prior[j] if torch.is_tensor(prior) else 0, diff[j])
                             for j in range(seg)]
                    total = sum(tp[0] for tp in parts) / seg
                    vals = sum(tp[1] for tp in parts) / seg
                elif dur.device.type == "cuda":
                    total, vals = OPS.loss_sum(dur, prior, diff)
                else:
                    total = dur + prior + diff
                    vals = torch.stack([dur.detach(), torch.as_tensor(prior).detach(), diff.detach(),
                                        total.detach()]).float()
                logged = vals if logged is None else logged + vals
                if i == n - 1 and self._arm is not None:
                    # the last micro-batch's backward exchanges the accumulated gradients (and the logged
                    # means) bucket by bucket as backward produces them ("local": pack only, no collective)
                    self.reducer.arm(logged / n, overlap=self._arm is True, comm=self._arm != "local")
                d = div if div is not None else n
                (total / d if d > 1 else total).backward()
        return logged / n if n > 1 else logged

    def _clip_and_update(self):
        if isinstance(self.optimizer, _FlatClipAdamW):  # graph mode: clipping is inside the fused step
            self.optimizer.step()
            return
        if self.cfg.gradient_clip_val:
            torch.nn.utils.clip_grad_norm_(self.params, self.cfg.gradient_clip_val, foreach=True)
        self.optimizer.step()

    def _group_stacked(self, order):
        """The recorded backward order with the weights that one stacked GEMM produces (q|k|v of the decoder's
        attention and of the text encoder's) placed back to back in stacking order, so that their flat-buffer
        views form one region the stacked weight-gradient GEMM writes in place (_ops._grad_buf_stacked)."""
        groups = []
        for m in self.model.modules():
            for names in (("to_q", "to_k", "to_v"), ("query_conv", "key_conv", "value_conv")):
                if all(isinstance(getattr(m, n, None), torch.nn.Module) for n in names):
                    groups.append([getattr(m, n).weight for n in names])
        member = {id(p): g for g in groups for p in g}
        present = {id(p) for p in order}
        out, done = [], set()
        for p in order:
            g = member.get(id(p))
            if g is not None and all(id(q) in present for q in g):
                if id(p) not in done:
                    out.extend(g)
                    done.update(id(q) for q in g)
            else:
                out.append(p)
        return out

    def _ensure_reducer(self, batches, run_step):
        """First DP step: one pass with an arrival recorder fixes the bucket layout (backward order)."""
        if self.reducer is not None:
            return None
        from matcha import dp as DP

        rec = DP.ArrivalRecorder(self.params)
        try:
            logged = run_step()
        finally:
            rec.remove()
        order = self._group_stacked(rec.order)
        if self.world > 1:  # one bucket layout on every rank: rank 0's recorded backward order
            index = {id(p): i for i, p in enumerate(self.params)}
            box = [[index[id(p)] for p in order]]
            dist.broadcast_object_list(box, src=0, group=self._host_group)
            if sorted(box[0]) != sorted(index[id(p)] for p in order):
                raise RuntimeError("data parallel: the ranks differentiate different parameter sets")
            order = [self.params[i] for i in box[0]]
        comm = DP.make_comm(self.dev, self.cfg.comm)
        seams, mb = (), self.cfg.bucket_mb
        enc = getattr(self.model, "encoder", None)
        if self.cfg.bucket_seams and self.cfg.graph and isinstance(enc, torch.nn.Module):
            enc_ids = {id(p) for p in enc.parameters()}
            first_enc = next((p for p in order if id(p) in enc_ids), None)
            if first_enc is not None:
                seams, mb = (first_enc,), max(mb, self.cfg.seam_bucket_mb)
        self.reducer = DP.GradBucketReducer(order, comm, mb, self.dev, seams=seams)
        self.reducer.watchdog, self.reducer.progress = self.watchdog, self.progress
        if isinstance(self.optimizer, _FlatClipAdamW):  # the mean over ranks rides in the fused optimizer step
            self.optimizer.grad_scale = comm.post_scale
            self.reducer.grad_scale_applied = True
        if comm.capturable:
            self.reducer.warm()  # every rank, now: later captures run without any collective
        return logged

    # ------------------------------------------------------------------------------------ eager
    def _eager_step(self, batches):
        n = len(batches)
        ddp = self.dp_mode == "ddp"

        def sync_ctx(i):
            return self.wrapped.no_sync() if (ddp and i < n - 1) else contextlib.nullcontext()

        if self.dp_mode == "buckets" and self.reducer is None:
            logged = self._ensure_reducer(batches, lambda: self._fwd_bwd(batches))
            # this first step: pack what backward produced and reduce it in one call
            for i, p in enumerate(self.reducer.params):
                self.reducer.views[i].copy_(p.grad)
            self.reducer.flat[self.reducer.n_grad:].copy_(logged)
            self.reducer.reduce_now()
            self.reducer.attach_views()
            logged = self.reducer.scalars().clone()
        elif self.dp_mode == "buckets":
            self._arm = True
            try:
                self._fwd_bwd(batches)
            finally:
                self._arm = None
                OPS.set_grad_slots(None)  # an aborted backward leaves no slots armed
            self.reducer.finish()
            logged = self.reducer.scalars().clone()
        else:
            logged = self._fwd_bwd(batches, sync_ctx)
            if ddp:  # the step's logged scalars in one collective (sync_dist=True)
                dist.all_reduce(logged)
                logged = logged / self.world
        self._clip_and_update()
        if self.progress is not None and self.dev.type == "cuda":
            self.progress.mark_step(torch.cuda.current_stream(self.dev))
        self.optimizer.zero_grad(set_to_none=True)
        return logged

    # ------------------------------------------------------------------------------------ graph
    def _graph_capture(self, batches):
        """Captures the step for this input-shape key.  N=1: graph 1 = fwd+bwd (fresh gradients),
        graph 2 = clip + AdamW on them.  DP with a capturable communicator: ONE graph -- fwd, bwd with
        each bucket's RCCL all-reduce forked off as backward completes it, join, clip + AdamW on the
        reduced flat buffer.  DP with torch.distributed: graph 1 packs the buckets, the host reduces
        the flat buffer, graph 2 steps."""
        e = {"static": [{k: v.clone() for k, v in b.items()} for b in batches]}
        static = e["static"]
        # warm-up (allocator pools, lazy library loads, optimizer state) must not leave updates behind
        saved = [p.detach().clone() for p in self.params]
        saved_state = self.optimizer.state_snapshot()
        side = torch.cuda.Stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            # warm-up passes are rank-local (no collective): a rank may capture a new shape while its peers
            # replay; only the first step of all (the reducer's construction) communicates, on every rank
            for it in range(2):
                for p in self.params:
                    p.grad = None
                if self.dp and self.reducer is None:
                    self._ensure_reducer(batches, lambda: self._fwd_bwd(static))
                    for i, p in enumerate(self.reducer.params):
                        self.reducer.views[i].copy_(p.grad)
                    self.reducer.attach_views()
                elif self.dp:
                    self._arm = "local"
                    try:
                        self._fwd_bwd(static)
                    finally:
                        self._arm = None
                        OPS.set_grad_slots(None)  # an aborted backward leaves no slots armed
                    self.reducer.finish()
                else:
                    self._fwd_bwd(static)
                self._clip_and_update()
        torch.cuda.current_stream(self.dev).wait_stream(side)
        gparams = [p for p in self.params if p.grad is not None]  # parameters the step differentiates
        with torch.no_grad():
            for p, s_ in zip(self.params, saved):
                p.copy_(s_)
            self.optimizer.state_restore(saved_state)  # moments / step back to their pre-warm-up values

        overlap = self.dp and self.reducer.comm.capturable
        if self.dp:
            self.reducer.attach_views()
            self.optimizer.bind_grads()  # the table points at the flat buffer's views (fixed addresses)
        # with a process group up, its watchdog thread polls the events of earlier collectives (e.g. the
        # eager all-reduce of the torch.distributed transport) at any time; in the default "global"
        # capture mode such a query from another thread invalidates the capture and aborts the
        # process.  "thread_local" restricts only this thread (the autograd thread's launches still go
        # to the capturing stream and its allocations to the graph pool)
        mode = "thread_local" if (dist.is_available() and dist.is_initialized()) else "global"
        e["g_fb"] = torch.cuda.CUDAGraph()
        with torch.cuda.graph(e["g_fb"], capture_error_mode=mode):
            for p in self.params:
                p.grad = None  # autograd hands over each fresh gradient: no accumulate kernels
            if self.dp:
                self._arm = overlap
                try:
                    e["logged"] = self._fwd_bwd(static)
                finally:
                    self._arm = None
                    OPS.set_grad_slots(None)  # an aborted backward leaves no slots armed
                self.reducer.finish()  # joins the forked all-reduces; .grad -> flat views
                if overlap:
                    self._clip_and_update()
                    if self.progress is not None:  # the device's "step done" marker, a node of the graph
                        self.progress.mark_step(torch.cuda.current_stream(self.dev))
            else:
                e["logged"] = self._fwd_bwd(static)
        e["fb_grads"] = [p.grad for p in gparams]  # graph-pool outputs, kept alive with the graph
        e["g_opt"] = None
        if not overlap:
            if not self.dp:  # the optimizer graph's table points at the (fixed) graph-pool gradients
                self.optimizer.bind_grads()
            e["g_opt"] = torch.cuda.CUDAGraph()
            with torch.cuda.graph(e["g_opt"], pool=e["g_fb"].pool(), capture_error_mode=mode):
                self._clip_and_update()
        e["opt_keep"] = (self.optimizer._table, self.optimizer._ws)  # the captured kernels read these
        e["overlap"] = overlap
        return e

    def _agree_shapes(self, batches):
        """TrainConfig.agree_shapes (N>1 graph step, ON by default): MAX over ranks of each micro-batch's padded Tx /
        Ty (and one batch size), then zero padding up to it, so every rank looks up the same key.  The padded
        frames are masked, but the decoder's arithmetic depends on the padded length (GroupNorm statistics
        over the whole padded length, conv bias leaking into padded frames -- SURVEY 0.6), so with the default a
        rank's losses depend on its peers' padded lengths (tests/test_distributed_cpu.py measures the difference
        against per-rank padding); agree_shapes=False keeps each rank's own padding, as the reference's DDP
        would."""
        if not (self.cfg.agree_shapes and self.dp and self.world > 1 and self.cfg.graph):
            return batches
        dims = torch.tensor([[b["x"].shape[1], b["y"].shape[2], b["x"].shape[0], -b["x"].shape[0]] for b in batches],
                            dtype=torch.int64)
        dist.all_reduce(dims, op=dist.ReduceOp.MAX, group=self._host_group)
        out = []
        for b, (tx, ty, bmax, nbmin) in zip(batches, dims.tolist()):
            if bmax != -nbmin:
                raise ValueError(f"data parallel graph step: per-rank batch sizes differ ({-nbmin}..{bmax})")
            b = dict(b)
            if b["x"].shape[1] < tx:
                b["x"] = torch.nn.functional.pad(b["x"], (0, tx - b["x"].shape[1]))
            if b["y"].shape[2] < ty:
                b["y"] = torch.nn.functional.pad(b["y"], (0, ty - b["y"].shape[2]))
                if "z" in b:
                    b["z"] = torch.nn.functional.pad(b["z"], (0, ty - b["z"].shape[2]))
            out.append(b)
        return out

    def _graph_step(self, batches):
        batches = self._agree_shapes(batches)
        key = tuple(tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(b.items())) for b in batches)
        if self.watchdog is not None:
            self.watchdog.note(graph_key="|".join(f"B{b['x'].shape[0]}xTx{b['x'].shape[1]}xTy{b['y'].shape[-1]}"
                                                  for b in batches), graph_cached=key in self._graphs)
        e = self._graphs.get(key)
        if e is None:
            e = self._graph_capture(batches)
            self._graphs[key] = e
            while len(self._graphs) > max(1, self.cfg.graph_cache):
                self._graphs.popitem(last=False)  # least recently used shape
        else:
            self._graphs.move_to_end(key)
        for b, s in zip(batches, e["static"]):
            for k, v in s.items():
                if b[k] is not v:
                    v.copy_(b[k], non_blocking=True)
        e["g_fb"].replay()
        if not self.dp:
            e["g_opt"].replay()
            return e["logged"]
        if not e["overlap"]:  # torch.distributed transport: one eager all-reduce of the packed buffer
            self.reducer.reduce_now()
            e["g_opt"].replay()
            if self.progress is not None:
                self.progress.mark_step(torch.cuda.current_stream(self.dev))
        return self.reducer.scalars().clone()  # the flat buffer is overwritten by the next replay

    def measure_dp_tail(self, batches) -> dict | None:
        """The data-parallel step's exposed tail: ONE extra eager forward + backward with the
        reducer armed exactly as in the graph step (every rank calls it together; no optimizer update, results
        discarded), with HIP events on the main stream at the end of the backward and on the reducer stream
        around the last bucket's pack + all-reduce.  Returns the all-reduce's own time and the part of it the
        main stream waits for (exposed = end of the last all-reduce - end of the backward, >= 0).  None unless a
        capturable (RCCL) reducer runs on a GPU."""
        r = self.reducer
        if r is None or not self.dp or self.dev.type != "cuda" or not r.comm.capturable:
            return None
        ev = {k: torch.cuda.Event(enable_timing=True) for k in ("start", "end", "bwd_end")}
        r.tail_events = ev
        for p in self.params:
            p.grad = None
        self._arm = True
        try:
            self._fwd_bwd(self._agree_shapes(batches))
        finally:
            self._arm = None
            OPS.set_grad_slots(None)
            r.tail_events = None
        r.finish()
        torch.cuda.synchronize(self.dev)
        ar = ev["start"].elapsed_time(ev["end"])
        exposed = max(0.0, ev["bwd_end"].elapsed_time(ev["end"]))
        return {"tail_bucket": len(r.buckets) - 1, "tail_bucket_mb": round((r.spans[-1][1] - r.spans[-1][0]) * 4 / 2 ** 20, 3),
                "tail_pack_allreduce_us": round(ar * 1e3, 1), "tail_exposed_us": round(exposed * 1e3, 1),
                "note": "one eager fwd+bwd after the timed region, reducer armed as in the graph step: HIP events "
                        "around the last bucket's pack + all-reduce (reducer stream) and at the backward's end "
                        "(main stream); exposed = all-reduce end - backward end"}

    # ------------------------------------------------------------------------------------ api
    def step(self, batches: list[dict]) -> torch.Tensor:
        """One optimizer step over len(batches) == accumulate_grad_batches micro-batches.  Returns the
        device tensor [dur, prior, diff, total] (mean over micro-batches and ranks); nothing here
        synchronises with the host."""
        assert len(batches) == self.cfg.accumulate_grad_batches
        if self.watchdog is not None:
            self.watchdog.beat(step_enqueueing=self.global_step)
        logged = self._graph_step(batches) if self.cfg.graph else self._eager_step(batches)
        self.global_step += 1
        self.last_losses = logged
        if self.watchdog is not None:
            self.watchdog.beat(last_step_enqueued=self.global_step - 1)
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
