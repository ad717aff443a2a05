"""The N>1 data-parallel path of matcha.training.Trainer on CPU with gloo (world size 2): replicas
start identical, each rank trains on its own shard, the gradient exchange makes every rank apply the
same update, equal to one process applying the mean of the per-rank gradients; the logged losses are
averaged across ranks in one collective."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class TinyTTS(torch.nn.Module):
    """Stand-in with MatchaTTS's forward interface and BaseLightningClass.configure_optimizers."""

    out_size = None

    def __init__(self):
        super().__init__()
        self.emb = torch.nn.Embedding(150, 16)
        self.proj = torch.nn.Linear(16, 80)

    def forward(self, x, x_lengths, y, y_lengths, out_size=None, cond=None, durations=None):
        mu = self.proj(self.emb(x)).mean(1)  # [B, 80]
        tgt = y.mean(-1)
        dur = (mu ** 2).mean() * 0.1
        prior = ((mu - tgt) ** 2).mean()
        diff = (mu.abs()).mean() * 0.01
        return dur, prior, diff, None

    def configure_optimizers(self):
        from matcha.models.baselightningmodule import BaseLightningClass

        return BaseLightningClass.configure_optimizers(self)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _batches(rank, accumulate):
    from matcha.training import synthetic_batch

    return [synthetic_batch(4, 12, 40, seed=100 * (m + 1) + rank, device="cpu") for m in range(accumulate)]


def _worker(rank, world, port, q, dp, accumulate, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(rank)  # different init per rank: the trainer must broadcast rank 0's weights
    from matcha.training import TrainConfig, Trainer

    model = TinyTTS()
    # bucket_mb tiny: TinyTTS's parameters fall into two buckets
    tr = Trainer(model, TrainConfig(precision="32-true", graph=False, dp=dp, accumulate_grad_batches=accumulate,
                                    bucket_mb=0.001))
    logs = []
    for _ in range(steps):
        logs.append(tr.step(_batches(rank, accumulate)).detach().clone().numpy())
    nb = len(tr.reducer.buckets) if tr.reducer is not None else 0
    state = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}  # by value, not fd-shared
    q.put((rank, state, logs, nb))
    dist.barrier()
    dist.destroy_process_group()


def _reference_update(accumulate, steps):
    """One process: rank 0's init; per step the mean over ranks of each rank's accumulated gradient
    (sum over micro-batches of grad(loss / accumulate)), clip_grad_norm_(1.0), AdamW."""
    torch.manual_seed(0)
    model = TinyTTS()
    opt = model.configure_optimizers()["optimizer"]
    logs = []
    for _ in range(steps):
        grads, losses = [], []
        for r in range(2):
            model.zero_grad(set_to_none=True)
            lr_ = 0
            for b in _batches(r, accumulate):
                d, p, f, _ = model(b["x"], b["x_lengths"], b["y"], b["y_lengths"])
                ((d + p + f) / accumulate).backward()
                lr_ = lr_ + torch.stack([d, p, f, d + p + f]).detach()
            grads.append([q.grad.clone() for q in model.parameters()])
            losses.append(lr_ / accumulate)
        for q, g0, g1 in zip(model.parameters(), *grads):
            q.grad = (g0 + g1) / 2
        torch.nn.utils.clip_grad_norm_(list(model.parameters()), 1.0)
        opt.step()
        logs.append((losses[0] + losses[1]) / 2)
    return {k: v.detach().clone() for k, v in model.state_dict().items()}, logs


@pytest.mark.timeout(180)
@pytest.mark.parametrize("dp,accumulate,steps", [("ddp", 1, 1), ("buckets", 1, 3), ("buckets", 2, 2)])
def test_data_parallel_two_ranks_gloo(dp, accumulate, steps):
    """ddp: torch DDP (the eager default).  buckets: matcha.dp.GradBucketReducer -- the flat, bucketed
    exchange the captured graph step uses (here eager over gloo): bucket layout from the recorded
    backward order, per-bucket packing from post-accumulate hooks, the logged means riding in the last
    bucket, .grad re-pointed at the flat buffer's views for the optimizer; step 1 records and reduces
    in one call, later steps issue each bucket as backward completes it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, dp, accumulate, steps)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, state, logs, nb = q.get(timeout=150)
        res[rank] = ({k: torch.from_numpy(v) for k, v in state.items()}, [torch.from_numpy(v) for v in logs], nb)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if dp == "buckets":
        assert res[0][2] >= 2  # several buckets actually exercised
    ref_state, ref_logs = _reference_update(accumulate, steps)
    for k in ref_state:
        torch.testing.assert_close(res[0][0][k], res[1][0][k], rtol=0, atol=0)  # replicas identical
        torch.testing.assert_close(res[0][0][k], ref_state[k], rtol=1e-5, atol=1e-7)
    for r in (0, 1):
        for got, want in zip(res[r][1], ref_logs):
            torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-7)


def _agree_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    torch.manual_seed(0)
    tr = Trainer(TinyTTS(), TrainConfig(precision="32-true", graph=True, accumulate_grad_batches=2, agree_shapes=True))
    # rank r: micro-batch shapes (Tx, Ty) differ per rank and per micro-batch
    shapes = {0: [(12, 40), (9, 48)], 1: [(10, 44), (11, 32)]}[rank]
    batches = [synthetic_batch(4, tx, ty, seed=rank * 10 + i, device="cpu") for i, (tx, ty) in enumerate(shapes)]
    for b in batches:
        b["z"] = torch.randn(4, 80, b["y"].shape[2])
    out = tr._agree_shapes(batches)
    got = [(tuple(b["x"].shape), tuple(b["y"].shape), tuple(b["z"].shape)) for b in out]
    same = all(torch.equal(o["x"][:, :b["x"].shape[1]], b["x"]) and torch.equal(o["y"][..., :b["y"].shape[2]], b["y"])
               and int(o["x"][:, b["x"].shape[1]:].abs().sum()) == 0 and float(o["y"][..., b["y"].shape[2]:].abs().sum()) == 0
               and torch.equal(o["x_lengths"], b["x_lengths"]) for o, b in zip(out, batches))
    # different batch sizes across ranks are refused (they could never share a captured graph)
    bad = [synthetic_batch(4 + rank, 8, 16, seed=1, device="cpu")] * 2
    try:
        tr._agree_shapes(bad)
        refused = False
    except ValueError:
        refused = True
    q.put((rank, got, same, refused))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_graph_step_shape_agreement_two_ranks_gloo():
    """Trainer._agree_shapes (the N>1 graph step with TrainConfig.agree_shapes): every rank pads each micro-batch to the MAX padded
    Tx / Ty over ranks with zeros (lengths unchanged), so all ranks look up, capture and replay one key."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, s, f)) for r, g, s, f in (q.get(timeout=100) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [((4, 12), (4, 80, 44), (4, 80, 44)), ((4, 11), (4, 80, 48), (4, 80, 48))]
    for r in (0, 1):
        assert res[r][0] == want, res[r][0]
        assert res[r][1] and res[r][2]


def test_bucket_layout_cuts_at_seams():
    """GradBucketReducer(seams=...): a bucket boundary at every seam parameter (the Trainer passes the text
    encoder's first-arriving parameter, so the decoder's gradients are issued together at the decoder / encoder
    seam of the backward), the usual size cuts inside each part, the small tail bucket last."""
    from matcha.dp import GradBucketReducer

    ps = [torch.zeros(1000, requires_grad=True) for _ in range(10)]
    r = GradBucketReducer(ps, None, bucket_mb=1.0, device=torch.device("cpu"), tail_mb=0.005, seams=[ps[6]])
    assert r.buckets[0][0] == 0 and r.buckets[-1][1] == 10
    assert all(b[1] == c[0] for b, c in zip(r.buckets, r.buckets[1:]))  # contiguous
    assert not any(s < 6 < e for s, e in r.buckets) and any(s == 6 for s, _ in r.buckets)
    assert r.buckets[-1][1] - r.buckets[-1][0] == 2  # tail: the last 8 KB (>= 5 KB)
    plain = GradBucketReducer(ps, None, bucket_mb=1.0, device=torch.device("cpu"), tail_mb=0.005)
    assert any(s < 6 < e for s, e in plain.buckets)
    r.remove()
    plain.remove()
