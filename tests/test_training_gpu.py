"""Train-step driver on the GPU: the captured-graph step equals the eager step (dropout off), replays
draw fresh dropout masks, and losses stay finite over a few steps."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _model(seed=0):
    from matcha.models.matcha_tts import MatchaTTS

    torch.manual_seed(seed)
    return MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)


@pytest.mark.parametrize("precision", ["32-true", "bf16-mixed"])
def test_graph_step_matches_eager_step(precision):
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    b = synthetic_batch(4, 20, 80, device=DEV)
    m1, m2 = _model(), _model()
    m2.load_state_dict(m1.state_dict())
    m1.eval()  # dropout off: both modes must then compute the same update
    m2.eval()
    t = torch.rand(4, 1, 1, device=DEV)
    z = torch.randn(4, 80, 80, device=DEV)
    for m in (m1, m2):  # inject the CFM randomness identically (MatchaTTS.forward's fused-loss entry)
        m.decoder.compute_loss_and_prior = (lambda f: (lambda *a, **k: f(*a, **{**k, "t": t, "z": z})))(
            m.decoder.compute_loss_and_prior)
    te = Trainer(m1, TrainConfig(precision=precision, graph=False))
    tg = Trainer(m2, TrainConfig(precision=precision, graph=True))
    le = te.step([b]).clone()
    lg = tg.step([b]).clone()
    torch.cuda.synchronize()
    # same weights -> same losses.  fp32: 1e-5.  bf16: library kernels outside libmtts (torch SDPA under
    # autocast, MIOpen encoder convs) may select other algorithms under stream capture, and bf16 rounding
    # amplifies that; the north-star loss tolerance (1e-4 relative) applies.
    rtol = 1e-5 if precision == "32-true" else 1e-4
    torch.testing.assert_close(lg, le, rtol=rtol, atol=1e-6)
    for _ in range(2):
        te.step([b])
        tg.step([b])
    torch.cuda.synchronize()
    # torch's embedding backward (text encoder) accumulates with atomics, and AdamW turns tiny
    # gradient differences into steps of up to ~lr each: a near-zero gradient whose sign differs moves
    # the two copies apart by at most 2*lr per step -> 3 steps * 2 * 1e-4
    for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        assert (p2 - p1).abs().max().item() <= 6e-4, n
    p0 = dict(_model().named_parameters())
    moved = [(p1 - p0[n]).abs().max().item() for n, p1 in m1.named_parameters()]
    assert max(moved) > 1e-5  # the optimizer actually stepped


def test_graph_replays_draw_new_dropout_masks():
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    b = synthetic_batch(4, 20, 80, device=DEV)
    m = _model(1)
    m.train()
    tr = Trainer(m, TrainConfig(precision="bf16-mixed", graph=True))
    losses = torch.stack([tr.step([b]).clone() for _ in range(4)])
    torch.cuda.synchronize()
    assert torch.isfinite(losses).all()
    assert len({round(v, 6) for v in losses[:, 2].tolist()}) > 1  # diff loss changes (t, z, masks)


def test_side_stream_wgrad_matches_main_stream():
    """Weight gradients launched on the side stream (components/_ops.py side_stream_wgrad) equal the
    main-stream ones: same kernels, same inputs -- only the ordering against the dgrad chain moves."""
    from matcha.models.components import _ops as OPS
    from matcha.training import synthetic_batch

    b = synthetic_batch(4, 20, 80, device=DEV)
    m = _model(2)
    m.eval()
    t = torch.rand(4, 1, 1, device=DEV)
    z = torch.randn(4, 80, 80, device=DEV)

    def grads(side):
        m.zero_grad(set_to_none=True)
        with OPS.side_stream_wgrad(side):
            dur, prior, diff, _ = m(**b, t=t, z=z)
            (dur + prior + diff).backward()
        torch.cuda.synchronize()
        return {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}

    g0, g1 = grads(False), grads(True)
    assert g0.keys() == g1.keys() and len(g0) > 100
    for n in g0:  # the decoder runs on libmtts alone: bitwise.  The encoder's torch kernels (embedding
        if n.startswith("decoder."):  # backward with atomics, library convs) need not be deterministic
            assert torch.equal(g1[n], g0[n]), n
        else:
            torch.testing.assert_close(g1[n], g0[n], rtol=1e-4, atol=1e-6)


def test_deferred_grad_sums_match_immediate():
    """The batched, deferred parameter-gradient sums (csrc/reduce.hip) equal the per-layer ones bitwise
    on the decoder (same fixed-order sums, one launch instead of one per layer)."""
    from matcha.models.components import _ops as OPS
    from matcha.training import synthetic_batch

    b = synthetic_batch(4, 20, 80, device=DEV)
    m = _model(3)
    m.eval()
    t = torch.rand(4, 1, 1, device=DEV)
    z = torch.randn(4, 80, 80, device=DEV)

    def grads(defer):
        m.zero_grad(set_to_none=True)
        with OPS.deferred_grad_sums(defer):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                dur, prior, diff, _ = m(**b, t=t, z=z)
            (dur + prior + diff).backward()
            if defer:
                assert N.lib().mtts_pending_reductions() > 50  # queued, not yet run
        torch.cuda.synchronize()
        return {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}

    from matcha import _native as N

    g0, g1 = grads(False), grads(True)
    assert N.lib().mtts_pending_reductions() == 0
    assert g0.keys() == g1.keys() and len(g0) > 100
    for n in g0:
        if n.startswith("decoder."):
            assert torch.equal(g1[n], g0[n]), n
        else:
            torch.testing.assert_close(g1[n], g0[n], rtol=1e-4, atol=1e-6)
