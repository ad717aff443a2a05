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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(rank)  # different init per rank: DDP must broadcast rank 0's weights
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    model = TinyTTS()
    tr = Trainer(model, TrainConfig(precision="32-true", graph=False))
    b = synthetic_batch(4, 12, 40, seed=100 + rank, device="cpu")
    logged = tr.step([b])
    state = {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}  # by value, not fd-shared
    q.put((rank, state, logged.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def _reference_update():
    """One process: rank 0's init, mean of the two shards' gradients, one clip + AdamW step."""
    from matcha.training import synthetic_batch

    torch.manual_seed(0)
    model = TinyTTS()
    grads, losses = [], []
    for r in range(2):
        model.zero_grad(set_to_none=True)
        b = synthetic_batch(4, 12, 40, seed=100 + r, device="cpu")
        d, p, f, _ = model(b["x"], b["x_lengths"], b["y"], b["y_lengths"])
        (d + p + f).backward()
        grads.append([q.grad.clone() for q in model.parameters()])
        losses.append(torch.stack([d, p, f, d + p + f]).detach())
    for q, g0, g1 in zip(model.parameters(), *grads):
        q.grad = (g0 + g1) / 2
    torch.nn.utils.clip_grad_norm_(list(model.parameters()), 1.0)
    opt = model.configure_optimizers()["optimizer"]
    opt.step()
    return {k: v.detach().clone() for k, v in model.state_dict().items()}, (losses[0] + losses[1]) / 2


@pytest.mark.timeout(180)
def test_data_parallel_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, state, logged = q.get(timeout=150)
        res[rank] = ({k: torch.from_numpy(v) for k, v in state.items()}, torch.from_numpy(logged))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_state, ref_logged = _reference_update()
    for k in ref_state:
        torch.testing.assert_close(res[0][0][k], res[1][0][k], rtol=0, atol=0)  # replicas identical
        torch.testing.assert_close(res[0][0][k], ref_state[k], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(res[0][1], ref_logged, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(res[1][1], ref_logged, rtol=1e-5, atol=1e-7)
