"""The captured data-parallel step on the MI355X (matcha/dp.py, csrc/dp_comm.cpp), rehearsed on one GPU
with a world-size-1 process group (8-GPU runs are the driver's): the bucketed RCCL all-reduces issued
from post-accumulate hooks inside HIP stream capture (the overlapped path bench.py takes at N>1), and
the torch.distributed transport (pack in the graph, one eager all-reduce after it).  With one rank
the exchange is an identity, so both must reproduce the plain N=1 graph step bit for bit: same
losses, same parameters after several steps.  Also: the shape-keyed cache of captured steps."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _model(seed=0):
    from matcha.models.matcha_tts import MatchaTTS

    torch.manual_seed(seed)
    m = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
    m.eval()
    return m


def _inject(m, t, z):
    m.decoder.compute_loss_and_prior = (lambda f: (lambda *a, **k: f(*a, **{**k, "t": t, "z": z})))(
        m.decoder.compute_loss_and_prior)


@pytest.fixture
def world1():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=DEV)
    yield
    dist.destroy_process_group()


def _run(dp: bool, comm: str, steps: int, bucket_mb: float = 4.0):
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    b = synthetic_batch(4, 24, 96, seed=3, device=DEV)
    m = _model(11)
    t = torch.rand(4, 1, 1, generator=torch.Generator(device=DEV).manual_seed(1), device=DEV)
    z = torch.randn(4, 80, 96, generator=torch.Generator(device=DEV).manual_seed(2), device=DEV)
    _inject(m, t, z)
    old = Trainer.force_dp
    Trainer.force_dp = dp
    try:
        tr = Trainer(m, TrainConfig(graph=True, comm=comm, bucket_mb=bucket_mb))
    finally:
        Trainer.force_dp = old
    logs = [tr.step([b]).clone() for _ in range(steps)]
    torch.cuda.synchronize()
    return tr, torch.stack(logs), {n: p.detach().clone() for n, p in m.named_parameters()}


@pytest.mark.parametrize("comm", ["rccl", "torch"])
def test_graph_dp_step_equals_single_gpu_step(world1, comm):
    tr, logs, params = _run(True, comm, 3)
    assert tr.reducer is not None and len(tr.reducer.buckets) >= 3  # 4 MB buckets over 19 M parameters
    e = next(iter(tr._graphs.values()))
    assert e["overlap"] == (comm == "rccl")  # rccl: the all-reduces are inside the captured graph
    _, logs0, params0 = _run(False, "auto", 3)
    assert torch.equal(logs, logs0), (logs, logs0)
    for n in params0:
        assert torch.equal(params[n], params0[n]), n


def test_graph_cache_per_shape():
    """Bucketed batch shapes reuse their captured step (no recapture when a shape comes back); the
    cache is LRU-bounded by TrainConfig.graph_cache."""
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    m = _model(12)
    tr = Trainer(m, TrainConfig(graph=True, graph_cache=2))
    shapes = [(4, 20, 80), (4, 24, 96), (4, 20, 80), (4, 24, 96), (4, 16, 64)]
    captured = []
    for B, Tx, Ty in shapes:
        n0 = len(tr._graphs)
        keys0 = set(tr._graphs)
        tr.step([synthetic_batch(B, Tx, Ty, seed=Tx, device=DEV)])
        captured.append(set(tr._graphs) != keys0 or len(tr._graphs) != n0)
    torch.cuda.synchronize()
    assert captured == [True, True, False, False, True]
    assert len(tr._graphs) == 2
    assert torch.isfinite(tr.last_losses).all()
