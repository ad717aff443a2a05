"""Data-parallel gradient exchange of the training step: bucketed all-reduce overlapped with backward.

The reference trains on one device (train.py:81-84); the north star (BASELINE.json) shards
utterances over the GPUs of a node with the gradient all-reduce over RCCL overlapped with backward.
DDP does that eagerly; the captured training step (matcha/training.py, graph=True) needs the
collectives INSIDE its HIP graph, which torch's ProcessGroupNCCL cannot provide on this stack
(tools/graph_event_probe.py: its watchdog aborts the process during capture), so:

* ``GradBucketReducer`` lays every differentiated parameter's gradient out in one flat fp32 buffer,
  in the order backward produces them (recorded in a warm-up pass), cut into ~``bucket_mb`` buckets.
  The armed backward writes the gradients of the conv / linear / FeedForward weights straight into their
  flat views (``_ops.set_grad_slots``: the producers allocate their output there, AccumulateGrad adopts
  it as ``.grad``).  A post-accumulate-grad hook counts each bucket's gradients; when the last one lands,
  the queued weight-gradient GEMMs / sums that produce them are flushed onto the deferral's side stream and
  the bucket is packed (one multi-tensor copy of the gradients that are not already in place -- norms,
  embeddings, the time MLP) and reduced on the reducer's stream after
  both the main and the side stream -- captured, that is a forked branch of the graph, so the reduction
  of bucket k runs while backward computes bucket k+1, and the main stream never waits for the side
  stream's weight gradients (the N=1 step's decoder / encoder seam overlap is kept).
  Buckets are issued strictly in index order on every rank (RCCL requires one collective order).
  The step's logged scalars ride in the last bucket: one collective for everything
  (baselightningmodule.py:117-199 issues one sync_dist all-reduce per logged value).
* ``RcclComm``: an RCCL communicator owned by libmtts_hip (csrc/dp_comm.cpp, include/mtts_dp.h)
  whose ``ncclAllReduce(ncclAvg)`` may be captured.  ``TorchComm``: torch.distributed (gloo on CPU,
  or any backend eagerly); it cannot be captured, so a graph step with it reduces the whole flat
  buffer once after the graph (no overlap) -- the shared-GPU gloo rehearsal uses that.

Gradient averaging (mean over ranks, DDP's semantics) happens before clipping: TorchComm sums then divides;
RcclComm SUMS (ncclSum) and leaves the factor ``post_scale = 1 / world`` to the consumer -- the Trainer's
fused clip + AdamW multiplies by it (``mtts_clip_adamw_scaled``: exact for a power-of-two world, so the
update equals the ncclAvg one bit for bit), any other consumer gets the flat buffer scaled in place by
``finish()``.  So with RcclComm under the Trainer's graph step, each parameter's ``.grad`` after the step holds
the SUM over ranks, not DDP's mean (``GradBucketReducer.grad_scale_applied``; ``mean_grads()`` returns the
means): anything that reads ``.grad`` after a step (norm logging, comparisons with DDP) must use that.  Why: RCCL's ncclAvg is a pre-multiply-sum, and at one rank it still launches a read-modify-write
kernel over the whole 76 MB buffer (oneRankReduce, ~143 us of the forced-DP N=1 step, profiles/r05/dp/);
an in-place ncclSum at one rank launches nothing.
"""
from __future__ import annotations

import contextlib
import ctypes

import torch
import torch.distributed as dist

from matcha import _native as N

N.register("mtts_dp_unique_id", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t])
N.register("mtts_dp_comm_init", ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.POINTER(ctypes.c_void_p)])
N.register("mtts_dp_allreduce_f32", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                                   ctypes.c_void_p])
N.register("mtts_dp_comm_query", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                                ctypes.POINTER(ctypes.c_int32)])
N.register("mtts_dp_comm_destroy", ctypes.c_int, [ctypes.c_void_p])
N.register("mtts_dp_rccl_version", ctypes.c_int, [])


class TorchComm:
    """torch.distributed all-reduce (sum, then / world): eager only."""

    capturable = False
    post_scale = 1.0  # all_reduce_ leaves the mean

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.ranks = self.world  # the ranks the collective spans
        self.backend = dist.get_backend(group)

    def all_reduce_(self, t: torch.Tensor) -> None:
        dist.all_reduce(t, group=self.group)
        t.div_(self.world)


class RcclComm:
    """One RCCL communicator for this process (ranks as torch.distributed's), capturable."""

    capturable = True

    def __init__(self, device: torch.device):
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        uid = (ctypes.c_char * 128)()
        if self.rank == 0:
            N.check(N.lib().mtts_dp_unique_id(uid, 128), "mtts_dp_unique_id")
        box = [bytes(uid)]
        dist.broadcast_object_list(box, src=0)  # over the default group's store/backend
        uid = (ctypes.c_char * 128).from_buffer_copy(box[0])
        self._comm = ctypes.c_void_p()
        with torch.cuda.device(device):
            N.check(N.lib().mtts_dp_comm_init(uid, 128, self.world, self.rank, ctypes.byref(self._comm)),
                    "mtts_dp_comm_init")
        n, me = ctypes.c_int32(), ctypes.c_int32()
        N.check(N.lib().mtts_dp_comm_query(self._comm, ctypes.byref(n), ctypes.byref(me)), "mtts_dp_comm_query")
        if (n.value, me.value) != (self.world, self.rank):
            raise RuntimeError(f"RCCL communicator spans {n.value} ranks as rank {me.value}; torch.distributed "
                               f"has {self.world} / {self.rank}")
        self.ranks = n.value  # as RCCL itself reports it (ncclCommCount)
        self.post_scale = 1.0 / self.world  # all_reduce_ leaves the SUM
        self.version = int(N.lib().mtts_dp_rccl_version())
        self.backend = "rccl"

    def all_reduce_(self, t: torch.Tensor) -> None:
        N.check(N.lib().mtts_dp_allreduce_f32(self._comm, t.data_ptr(), t.numel(), 0,
                                              torch.cuda.current_stream(t.device).cuda_stream),
                "mtts_dp_allreduce_f32")

    def close(self):
        if self._comm:
            N.lib().mtts_dp_comm_destroy(self._comm)
            self._comm = ctypes.c_void_p()


def make_comm(device: torch.device, kind: str = "auto"):
    """'rccl' (libmtts_hip's communicator), 'torch' (torch.distributed), 'auto' = rccl on an nccl
    (RCCL) default group, torch otherwise (gloo)."""
    if kind == "auto":
        kind = "rccl" if (device.type == "cuda" and dist.get_backend() == "nccl") else "torch"
    return RcclComm(device) if kind == "rccl" else TorchComm()


class GradBucketReducer:
    """Flat, bucketed gradient all-reduce (see the module docstring).

    params: the differentiated parameters in the order backward finishes them.  After ``finish()``
    every parameter's ``.grad`` is a view of the reduced flat buffer (the optimizer reads these) and
    ``scalars()`` returns the averaged logged values."""

    N_SCALARS = 4

    def __init__(self, params, comm, bucket_mb: float = 16.0, device=None, tail_mb: float = 4.0, seams=()):
        self.params = list(params)
        self.comm = comm
        self.device = device or self.params[0].device
        self.index = {id(p): i for i, p in enumerate(self.params)}
        # buckets are cut from the END of the arrival order: the last bucket (the first layers, whose
        # gradients backward finishes last) is the one whose reduction cannot overlap anything, so it
        # is kept small (tail_mb); the others are ~bucket_mb.  seams: parameters that start a new bucket
        # whatever the size (the Trainer passes the text encoder's first-arriving parameter: the decoder's
        # gradients then form their own bucket(s), issued at the decoder / encoder seam of the backward --
        # exactly where the N=1 step flushes the decoder's queued weight gradients onto the side stream)
        limit = max(int(bucket_mb * 2 ** 20 / 4), 1)
        tail = max(int(min(tail_mb, bucket_mb) * 2 ** 20 / 4), 1)
        seam_idx = sorted({self.index[id(p)] for p in seams if id(p) in self.index} - {0})
        bounds = [0] + seam_idx + [len(self.params)]
        cuts = []
        for seg_lo, seg_hi in reversed(list(zip(bounds[:-1], bounds[1:]))):
            end, size = seg_hi, 0
            for i in range(seg_hi - 1, seg_lo - 1, -1):
                size += self.params[i].numel()
                if size >= (tail if not cuts else limit) and i > seg_lo:
                    cuts.append((i, end))
                    end, size = i, 0
            cuts.append((seg_lo, end))
        self.buckets = [c for c in reversed(cuts) if c[1] > c[0]] or [(0, len(self.params))]  # (start, end)
        self.bucket_of = []
        for k, (s, e) in enumerate(self.buckets):
            self.bucket_of += [k] * (e - s)
        offs, off = [], 0
        for p in self.params:
            offs.append(off)
            off += p.numel()
        self.offsets = offs
        self.n_grad = off
        # the last bucket's slice also carries the logged scalars (one collective per step)
        self.flat = torch.zeros(off + self.N_SCALARS, dtype=torch.float32, device=self.device)
        self.spans = []
        for k, (s, e) in enumerate(self.buckets):
            lo = offs[s] if s < len(self.params) else off
            hi = (offs[e] if e < len(self.params) else off) + (self.N_SCALARS if k == len(self.buckets) - 1 else 0)
            self.spans.append((lo, hi))
        self.views = [self.flat[o:o + p.numel()].view_as(p) for p, o in zip(self.params, offs)]
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        self.armed = False
        self.overlap = True
        self._pending_scalars = None
        self._ready = [0] * len(self.buckets)
        self._issued = 0
        self.grad_refs = None  # the gradient tensors packed in the last armed pass
        # True: the optimizer applies comm.post_scale itself (Trainer + fused AdamW); False: finish() /
        # reduce_now() scale the flat buffer in place when the comm leaves sums
        self.grad_scale_applied = False
        self.copied = {}  # bucket -> shapes of the gradients its last pack copied (not written in place)
        # bench.py's N>1 path (matcha/watchdog.py): the host watchdog hears of every bucket issue; the device
        # marks each bucket's completed all-reduce (a graph node after it on the reducer stream)
        self.watchdog = None
        self.progress = None
        # measure_tail(): HIP events around the last bucket's pack + all-reduce on the reducer stream
        self.tail_events = None

    # -------------------------------------------------------------------- per step
    def arm(self, scalars: torch.Tensor, overlap: bool, comm: bool = True) -> None:
        """Call before the backward of the last micro-batch.  ``scalars``: the 4 logged values
        (already the micro-batch mean).  overlap=False packs only; the caller reduces after.  comm=False
        packs only and never communicates (a graph capture's warm-up passes: a rank may capture a new
        shape while its peers replay, so only replays may issue collectives)."""
        from matcha.models.components import _ops as OPS

        self.armed = True
        OPS.set_grad_slots({p.data_ptr(): v for p, v in zip(self.params, self.views)})
        capturing = self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()
        self.overlap = (comm and overlap and self.comm is not None and (self.comm.capturable or not capturing))
        self._pending_scalars = scalars
        self._ready = [0] * len(self.buckets)
        self._issued = 0
        self.grad_refs = [None] * len(self.params)

    def _on_grad(self, p) -> None:
        if not self.armed:
            return
        i = self.index[id(p)]
        self.grad_refs[i] = p.grad
        k = self.bucket_of[i]
        self._ready[k] += 1
        while self._issued < len(self.buckets):  # strictly in bucket order on every rank
            k = self._issued
            s, e = self.buckets[k]
            if self._ready[k] < e - s:
                break
            self._issue(k)
            self._issued += 1

    def _pack(self, k: int) -> None:
        s, e = self.buckets[k]
        dst, src = [], []
        for i in range(s, e):  # gradients written in place (grad slots) need no copy
            g, v = self.grad_refs[i], self.views[i]
            if g.data_ptr() != v.data_ptr():
                dst.append(v)
                src.append(g.view_as(v) if g.shape != v.shape else g)
        self.copied[k] = [self.params[i].shape for i in range(s, e)
                          if self.grad_refs[i].data_ptr() != self.views[i].data_ptr()]
        if dst:
            torch._foreach_copy_(dst, src)
        if k == len(self.buckets) - 1:
            self.flat[self.n_grad:].copy_(self._pending_scalars)

    def _issue(self, k: int) -> None:
        from matcha.models.components import _ops as OPS

        lo, hi = self.spans[k]
        if self.watchdog is not None:
            self.watchdog.note(bucket_issued=k, buckets=len(self.buckets))
        if self.overlap and self.stream is not None:
            # the bucket's weight gradients may still be queued: they run on the deferral's side stream
            # (joined at the deferral's exit); pack + all-reduce here wait for the main and the side stream
            side = OPS.flush_for_bucket()
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            if side is not None:
                self.stream.wait_stream(side)
            with torch.cuda.stream(self.stream):
                tail = self.tail_events is not None and k == len(self.buckets) - 1
                if tail:
                    self.tail_events["start"].record(self.stream)
                self._pack(k)
                self.comm.all_reduce_(self.flat[lo:hi])
                if tail:
                    self.tail_events["end"].record(self.stream)
                if self.progress is not None:
                    self.progress.mark_bucket(k, self.stream)
        else:
            OPS.flush_deferred_grad_sums()  # on the current stream (joins the side stream first)
            self._pack(k)
            if self.overlap:  # CPU (gloo): eager, in order
                self.comm.all_reduce_(self.flat[lo:hi])
        if self.watchdog is not None:
            self.watchdog.beat(bucket_returned=k)

    def warm(self) -> None:
        """One eager all-reduce per bucket span on every rank (all ranks call this together, when the
        reducer is built): RCCL sets up its connections for each message size on first use, which must not
        happen later inside one rank's graph capture while its peers replay."""
        for lo, hi in self.spans:
            self.comm.all_reduce_(self.flat[lo:hi])
        self.flat.zero_()

    def finish(self) -> None:
        """After the armed backward: every bucket issued, the current stream joined with the reductions
        (overlap) or the whole buffer reduced now (no overlap), parameters' .grad -> flat views."""
        if not self.armed:
            return
        from matcha.models.components import _ops as OPS

        self.armed = False
        OPS.set_grad_slots(None)
        if self._issued != len(self.buckets):
            # a parameter got no gradient on this rank.  Its peers issue every bucket, so the remaining
            # ones are issued here too (missing gradients as zeros) before raising: the ranks stay in
            # one collective sequence instead of blocking forever in unmatched all-reduces
            missing = [i for i, g in enumerate(self.grad_refs) if g is None]
            for i in missing:
                self.grad_refs[i] = torch.zeros_like(self.params[i])
            while self._issued < len(self.buckets):
                self._issue(self._issued)
                self._issued += 1
            if self.overlap and self.stream is not None:
                torch.cuda.current_stream(self.device).wait_stream(self.stream)
            raise RuntimeError(f"GradBucketReducer: {len(missing)} parameters got no gradient this step "
                               f"(first: index {missing[:3]}); the bucket layout assumes a fixed set")
        if self.overlap:
            if self.stream is not None:
                if self.tail_events is not None:  # the backward's end on the main stream, before the join
                    self.tail_events["bwd_end"].record(torch.cuda.current_stream(self.device))
                torch.cuda.current_stream(self.device).wait_stream(self.stream)
            self._post_scale()
        self.attach_views()

    def _post_scale(self) -> None:
        ps = getattr(self.comm, "post_scale", 1.0)
        if ps != 1.0 and not self.grad_scale_applied:
            self.flat[:self.n_grad].mul_(ps)

    def reduce_now(self) -> None:
        """No-overlap mode: one all-reduce of the packed buffer (eager, e.g. after a graph replay)."""
        self.comm.all_reduce_(self.flat)
        self._post_scale()

    def mean_grads(self) -> list:
        """The parameters' gradients as DDP's means over ranks (``.grad`` holds sums when the optimizer applies
        the 1 / world factor itself)."""
        ps = getattr(self.comm, "post_scale", 1.0)
        if ps == 1.0 or not self.grad_scale_applied:
            return list(self.views)
        return [v * ps for v in self.views]

    def attach_views(self) -> None:
        for p, v in zip(self.params, self.views):
            p.grad = v

    def scalars(self) -> torch.Tensor:
        """The averaged logged values: a VIEW of the flat buffer's tail when the comm leaves the mean (the next
        step overwrites it: callers that keep it clone it -- Trainer does), else the tail times post_scale."""
        ps = getattr(self.comm, "post_scale", 1.0)
        tail = self.flat[self.n_grad:]
        return tail if ps == 1.0 else tail * ps

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


class ArrivalRecorder:
    """Records the order in which backward finishes the parameters' gradients (post-accumulate hooks)."""

    def __init__(self, params):
        self.order = []
        self._seen = set()
        self._hooks = [p.register_post_accumulate_grad_hook(self._on) for p in params]

    def _on(self, p):
        if id(p) not in self._seen:
            self._seen.add(id(p))
            self.order.append(p)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


@contextlib.contextmanager
def stdout_to_stderr():
    """File descriptor 1 -> 2 for the duration: gloo's rendezvous prints "Rank r is connected to n peer
    ranks" on stdout, where bench.py's rank 0 prints exactly one JSON line."""
    import os
    import sys

    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
