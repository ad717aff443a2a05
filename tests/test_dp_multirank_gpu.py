"""Two data-parallel ranks of the REAL MatchaTTS graph step on the one MI355X of the test box (both ranks on
cuda:0 over gloo -- RCCL refuses two ranks on one device; the 8-GPU RCCL runs are the driver's).

Each rank trains on its own shard with the captured step (fwd + bwd, bucket packing from the
post-accumulate hooks, one all-reduce of the flat gradient buffer, captured clip + AdamW).  The ranks get
batches of DIFFERENT padded lengths and keep them (no shape agreement): each captures its own shape, and the
collective sequence stays one because capture warm-ups never communicate -- only replays do.  After 3 steps both replicas
must be identical and equal one process that applies the mean gradient: accumulate_grad_batches=2 over
the two shards (grad of total/2 per micro-batch == the rank mean, exactly, since halving is exact) +
clip_grad_norm_(1.0) + AdamW -- train.py:81-89, baselightningmodule.py:115-199."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, TX, STEPS = 4, 24, 3
TY = {0: 96, 1: 80}  # each rank keeps its own padded length


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard(rank, dev):
    """Rank r's batch, with the CFM randomness (t, z) injected so that both runs draw the same."""
    from matcha.training import synthetic_batch

    b = synthetic_batch(B, TX, TY[rank], seed=50 + rank, device=dev)
    g = torch.Generator(device="cpu").manual_seed(60 + rank)
    b["t"] = torch.rand(B, 1, 1, generator=g).to(dev)
    b["z"] = torch.randn(B, 80, TY[rank], generator=g).to(dev)
    return b


def _model(dev, seed):
    from matcha.models.matcha_tts import MatchaTTS

    torch.manual_seed(seed)
    m = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev)
    m.eval()  # no dropout: the two runs see identical arithmetic
    return m


def _pad_to(b, ty):
    """Trainer._agree_shapes' zero padding of a batch (and its injected z) to ty frames."""
    b = dict(b)
    for k in ("y", "z"):
        b[k] = torch.nn.functional.pad(b[k], (0, ty - b[k].shape[2]))
    return b


def _worker(rank, world, port, precision, q, agree=False):
    import sys

    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root / "matcha-tts-etu-upmc-ensam_amd"), str(root)]
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from matcha.training import TrainConfig, Trainer

        m = _model(dev, seed=rank)  # different init per rank: the Trainer broadcasts rank 0's weights
        tr = Trainer(m, TrainConfig(graph=True, precision=precision, bucket_mb=4.0, agree_shapes=agree))
        b = _shard(rank, dev)
        logs = [tr.step([b]).cpu() for _ in range(STEPS)]
        torch.cuda.synchronize()
        key = next(iter(tr._graphs))
        # by value (numpy), not fd-shared tensors: this process may be gone when the parent unpickles
        q.put((rank, {n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()}, torch.stack(logs).numpy(),
               tr.reducer.comm.ranks, len(tr.reducer.buckets), repr(key)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("precision,agree", [("bf16-mixed", False), ("bf16-mixed", True)])
def test_two_ranks_real_model_graph_step_equals_mean_gradient(precision, agree):
    """agree=False: each rank keeps its own padding (the reference's DDP semantics).  agree=True (the Trainer's
    default): every rank pads to the max padded length over ranks (Ty 96), so the result equals one
    process over the shards padded to 96; its distance from per-rank padding -- the cost of the default -- is
    measured and printed (the padded frames enter the decoder's GroupNorm statistics)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, precision, q, agree)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            rank, params, logs, ranks, nbuckets, key = q.get(timeout=240)
            res[rank] = ({n: torch.from_numpy(v) for n, v in params.items()}, torch.from_numpy(logs), ranks, nbuckets,
                         key)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert res[0][2] == res[1][2] == 2  # the communicator spans both ranks
    assert res[0][3] >= 3  # several buckets exercised
    assert (res[0][4] == res[1][4]) == agree  # own padded shapes, or one agreed shape

    # one process, the mean gradient: accumulate_grad_batches=2 over the two shards, each at its own length
    # (agree: both padded to the max, as the ranks did); micro-batches not merged, so each shard's backward runs
    # alone exactly as on its rank
    from matcha.training import TrainConfig, Trainer

    dev = torch.device("cuda:0")

    def one_process(pad):
        m = _model(dev, seed=0)
        tr = Trainer(m, TrainConfig(graph=True, precision=precision, accumulate_grad_batches=2,
                                    merge_micro_batches=False))
        b0, b1 = _shard(0, dev), _shard(1, dev)
        if pad:
            ty = max(TY.values())
            b0, b1 = _pad_to(b0, ty), _pad_to(b1, ty)
        lg = torch.stack([tr.step([b0, b1]).cpu() for _ in range(STEPS)])
        torch.cuda.synchronize()
        return {n: p.detach().cpu() for n, p in m.named_parameters()}, lg

    want, logs = one_process(agree)
    if agree:  # the default's cost against the reference's per-rank padding, measured
        own, own_logs = one_process(False)
        dl = ((logs - own_logs).abs() / own_logs.abs().clamp_min(1e-12)).max(0).values
        dp = max(((want[n] - own[n]).norm() / own[n].norm().clamp_min(1e-12)).item() for n in own)
        print(f"\nagree_shapes=True vs per-rank padding after {STEPS} steps: logged [dur, prior, diff, total] max rel "
              f"diff {[f'{v:.3e}' for v in dl.tolist()]}, max per-tensor parameter rel diff {dp:.3e}")
        assert torch.isfinite(dl).all()

    for n in want:
        assert torch.equal(res[0][0][n], res[1][0][n]), n  # replicas identical
        torch.testing.assert_close(res[0][0][n], want[n], rtol=1e-5, atol=1e-7, msg=n)
    for r in (0, 1):
        torch.testing.assert_close(res[r][1], logs, rtol=1e-5, atol=1e-7)
    # the parameters moved (3 AdamW steps at lr 1e-4): the comparison is not of the initial weights
    m0 = _model(dev, seed=0)
    moved = sum(not torch.equal(p.detach().cpu(), want[n]) for n, p in m0.named_parameters())
    assert moved > 0.9 * len(want)
