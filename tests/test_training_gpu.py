"""Train-step driver on the GPU: the captured-graph step equals the eager step (dropout off), replays
draw fresh dropout masks, the HIP clip + AdamW equals torch's, gradient accumulation over two
micro-batches equals the reference's loss / 2 + one optimizer step (train.py:87-88)."""
from __future__ import annotations

import math

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
    # same weights, same kernels, fixed-order sums everywhere (deterministic embedding backward too):
    # the first step's losses are bitwise equal in both precisions
    assert torch.equal(lg, le), (lg, le)
    for _ in range(2):
        te.step([b])
        tg.step([b])
    torch.cuda.synchronize()
    # eager runs torch's AdamW, graph the HIP one (equal to 2 ulp, test_clip_adamw_matches_torch).
    # Adam normalises each gradient by its own running RMS, so a parameter whose gradient is pure
    # rounding noise (a bias ahead of a GroupNorm has true gradient 0) takes steps of up to ~lr whose
    # sign follows the noise: the two copies may drift apart by <= 2 * lr per step there -> 3 * 2e-4
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
    for n in g0:  # every gradient comes from libmtts (incl. the embedding's fixed-order backward): bitwise
        assert torch.equal(g1[n], g0[n]), n


@pytest.mark.parametrize("side", [False, True, "inline", "cap", "enc_chunks"])
def test_deferred_grad_sums_match_immediate(side):
    """The deferred weight-gradient GEMMs (launched batched, csrc/conv_gemm.hip) and parameter-gradient sums
    (csrc/reduce.hip) equal the per-layer ones bitwise on the decoder (same row splits, same fixed-order
    sums, a few launches instead of one or two per layer); side: batches of them run on a side stream while
    the backward goes on (joined at the context exit); "inline": batches of 8 flushed on the main stream as
    they queue up (MTTS_INLINE_REDUCE_JOBS; the default flushes once, at the end)."""
    from matcha import _native as N
    from matcha.models.components import _ops as OPS
    from matcha.training import synthetic_batch

    inline = side == "inline"
    cap = side == "cap"  # batched weight-gradient launches on a capped grid (37 workgroups walk the blocks)
    side = side is True
    saved_inline, saved_enc = OPS._DEFER["inline"], OPS._ENC_SIDE_JOBS
    OPS._DEFER["side_on"], OPS._DEFER["chunk"], OPS._DEFER["inline"] = side, 8, (8 if inline else 0)
    # the encoder's chunked side flushes (default) would empty the queue the plain mode checks; "enc_chunks"
    # keeps them (every 16 sums) and checks only the bitwise equality
    OPS._ENC_SIDE_JOBS = 16 if side == "enc_chunks" else 0
    # queued weight gradients run batched with the batched split plan: the immediate pass takes the same
    # plan, so the comparison isolates the batching (one launch for many layers) and the deferral
    N.lib().mtts_wgrad_plan_mode(1)

    b = synthetic_batch(4, 20, 80, device=DEV)
    m = _model(3)
    m.eval()
    t = torch.rand(4, 1, 1, device=DEV)
    z = torch.randn(4, 80, 80, device=DEV)

    def grads(defer):
        m.zero_grad(set_to_none=True)
        N.lib().mtts_wgrad_flush_cap(37 if (cap and defer) else 0)
        with OPS.deferred_grad_sums(defer):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                dur, prior, diff, _ = m(**b, t=t, z=z)
            (dur + prior + diff).backward()
            if defer and not side and not inline and OPS._ENC_SIDE_JOBS == 0:
                assert N.lib().mtts_pending_reductions() > 50  # queued, not yet run
            if defer and inline:
                assert N.lib().mtts_pending_reductions() < 8  # flushed in batches during the backward
            if defer and side:
                assert OPS._DEFER["side_used"]  # some batches already launched on the side stream
        torch.cuda.synchronize()
        return {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}

    try:
        g0, g1 = grads(False), grads(True)
    finally:
        OPS._DEFER["side_on"], OPS._DEFER["chunk"], OPS._DEFER["inline"] = False, 24, saved_inline
        OPS._ENC_SIDE_JOBS = saved_enc
        N.lib().mtts_wgrad_plan_mode(0)
        N.lib().mtts_wgrad_flush_cap(0)
    assert N.lib().mtts_pending_reductions() == 0
    assert g0.keys() == g1.keys() and len(g0) > 100
    for n in g0:
        assert torch.equal(g1[n], g0[n]), n


@pytest.mark.parametrize("grad_scale", [10.0, 1e-3])  # global norm above / below gradient_clip_val = 1
def test_clip_adamw_matches_torch(grad_scale):
    """The graph step's optimizer (csrc/optim.hip mtts_clip_adamw over the flat parameter array) against
    torch: clip_grad_norm_(1.0) (train.py:88 gradient_clip_val) + AdamW(1e-4, (0.9, 0.999), eps 1e-8,
    wd 1e-6) (baselightningmodule.py:59-65), identical gradients, three steps: parameters within 2 ulp,
    moments within fp32 rounding."""
    from matcha.training import _FlatClipAdamW

    g = torch.Generator().manual_seed(5)
    shapes = [(256, 160, 3), (256,), (1000,), (7, 5), (1,), (80, 256, 1), (3,)]
    init = [torch.randn(s, generator=g) for s in shapes]
    grads = [[torch.randn(s, generator=g) * grad_scale / math.sqrt(len(shapes)) for s in shapes] for _ in range(3)]
    p_hip = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    p_ref = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    lr = torch.tensor(1e-4, device=DEV, dtype=torch.float64)
    opt = _FlatClipAdamW(p_hip, lr, 1.0)
    ref = torch.optim.AdamW(p_ref, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-6)
    for step in range(3):
        for p, gr in zip(p_hip, grads[step]):
            p.grad = gr.to(DEV).clone()
        for p, gr in zip(p_ref, grads[step]):
            p.grad = gr.to(DEV).clone()
        opt.step()
        norm = torch.nn.utils.clip_grad_norm_(p_ref, 1.0)
        ref.step()
        torch.cuda.synchronize()
        assert (norm.item() > 1.0) == (grad_scale > 1.0)
        for i, (a, b) in enumerate(zip(p_hip, p_ref)):
            d = (a.detach() - b.detach()).abs()
            r = d / _ulp2(b.detach())
            j = int(r.argmax())
            assert r.max() <= 1.0, (step, i, a.reshape(-1)[j].item(), b.reshape(-1)[j].item(), grads[step][i].reshape(-1)[j].item())
        m_ref = torch.cat([ref.state[p]["exp_avg"].reshape(-1) for p in p_ref])
        v_ref = torch.cat([ref.state[p]["exp_avg_sq"].reshape(-1) for p in p_ref])
        m_hip = torch.cat([opt.exp_avg[o:o + p.numel()] for p, o in zip(p_hip, opt.offsets)])
        v_hip = torch.cat([opt.exp_avg_sq[o:o + p.numel()] for p, o in zip(p_hip, opt.offsets)])
        # the clip coefficient (a norm summed in another order) may differ by an ulp, which moves every
        # clipped gradient -- and the moments built from it -- by an ulp of the gradient scale
        torch.testing.assert_close(m_hip, m_ref, rtol=1e-6, atol=4 * torch.finfo(torch.float32).eps * m_ref.abs().max().item())
        torch.testing.assert_close(v_hip, v_ref, rtol=1e-6, atol=4 * torch.finfo(torch.float32).eps * v_ref.abs().max().item())


def test_clip_norm_independent_of_gradient_alignment():
    """The clipped step is bit-identical whether the gradients are allocator-aligned tensors or
    unaligned views into one buffer (the data-parallel step's buckets): the norm's summation order
    depends on the values only (csrc/optim.hip adamw_sumsq_kernel)."""
    from matcha.training import _FlatClipAdamW

    g = torch.Generator().manual_seed(9)
    shapes = [(192, 80, 3), (5,), (1001,), (7, 5), (1,), (33, 3)]
    init = [torch.randn(s, generator=g) for s in shapes]
    grads = [torch.randn(s, generator=g) * 3.0 for s in shapes]  # norm well above 1: clipping active
    out = []
    for shift in (0, 1, 3):
        ps = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
        opt = _FlatClipAdamW(ps, torch.tensor(1e-4, device=DEV, dtype=torch.float64), 1.0)
        buf = torch.zeros(sum(x.numel() for x in grads) + 8, device=DEV)
        off = shift
        for p, gr in zip(ps, grads):
            view = buf[off:off + gr.numel()].view_as(gr)
            view.copy_(gr.to(DEV))
            p.grad = view if shift else gr.to(DEV).clone()
            off += gr.numel()
        opt.step()
        torch.cuda.synchronize()
        out.append(opt.flat.clone())
    assert torch.equal(out[0], out[1]) and torch.equal(out[0], out[2])


@pytest.mark.parametrize("world", [4, 8, 3])
def test_clip_adamw_grad_scale_is_the_rank_mean(world):
    """the data-parallel step hands the fused optimizer gradient SUMS over `world` ranks with
    grad_scale = 1 / world (matcha/dp.py RcclComm: ncclSum, the mean folded into mtts_clip_adamw_scaled).  For a
    power-of-two world that is bitwise the unscaled step on the mean gradients (g * 2^-k is exact); for world = 3
    the scale rounds, and the parameters stay within 2 ulp of the step on the fp32 means.  Three steps, clipping
    active and inactive."""
    from matcha.training import _FlatClipAdamW

    g = torch.Generator().manual_seed(13)
    shapes = [(256, 80, 3), (17,), (1003,), (1,)]
    init = [torch.randn(s, generator=g) for s in shapes]
    # per-rank gradients whose fp32 sum is exact (multiples of 2^-12 well inside 24 bits)
    ranks = [[[torch.round(torch.randn(s, generator=g) * sc * 4096) / 4096 for s in shapes] for _ in range(world)]
             for sc in (3.0, 0.01, 0.5)]
    runs = {}
    for mode in ("sum_scaled", "mean"):
        ps = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
        opt = _FlatClipAdamW(ps, torch.tensor(1e-4, device=DEV, dtype=torch.float64), 1.0)
        for step_grads in ranks:
            sums = [torch.stack([r[i] for r in step_grads]).sum(0) for i in range(len(shapes))]
            for p, s in zip(ps, sums):
                p.grad = (s if mode == "sum_scaled" else s / world).to(DEV).contiguous()
            opt.grad_scale = 1.0 / world if mode == "sum_scaled" else 1.0
            opt.step()
        torch.cuda.synchronize()
        runs[mode] = opt.flat.clone()
    a, b = runs["sum_scaled"], runs["mean"]
    if world & (world - 1) == 0:
        assert torch.equal(a, b)
    else:
        assert ((a - b).abs() / _ulp2(b)).max().item() <= 1.0


def _inject(m, t, z):
    m.decoder.compute_loss_and_prior = (lambda f: (lambda *a, **k: f(*a, **{**k, "t": t, "z": z})))(
        m.decoder.compute_loss_and_prior)


@pytest.mark.parametrize("graph", [False, True])
def test_accumulate_grad_batches_2_vs_torch(graph):
    """Trainer(accumulate_grad_batches=2) (train.py:87: two micro-batches, loss / 2 each, one optimizer
    step) against one fp32 process doing exactly that with torch: backward of (dur + prior + diff) / 2
    per micro-batch, clip_grad_norm_(1.0), torch.optim.AdamW with the reference's defaults.  Dropout
    off, t / z injected; the gradients are bitwise deterministic (HIP kernels with fixed-order sums,
    deterministic embedding backward), so the first step's losses are bitwise equal.  Eager mode runs
    the reference's own optimizer: parameters bitwise equal after 1 and 3 steps.  Graph mode runs the
    HIP clip + AdamW: within 2 ulp after one step; after three steps every parameter stays within 1e-6
    relative except, possibly, those whose gradient is pure rounding noise (a bias ahead of a
    GroupNorm has true gradient 0): Adam normalises it to steps of ~lr whose sign follows the noise,
    so those may differ by up to 3 lr."""
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    b1 = synthetic_batch(4, 24, 96, seed=1, device=DEV)
    b2 = synthetic_batch(4, 24, 96, seed=2, device=DEV)
    m_tr, m_ref = _model(7), _model(7)
    m_ref.load_state_dict(m_tr.state_dict())
    m_tr.eval()
    m_ref.eval()
    t = torch.rand(4, 1, 1, device=DEV)
    z = torch.randn(4, 80, 96, device=DEV)
    _inject(m_tr, t, z)
    _inject(m_ref, t, z)
    # merge_micro_batches=False: each micro-batch on fresh gradients (stashed, summed at the end) -- the
    # separate micro-batches of the reference, bitwise
    tr = Trainer(m_tr, TrainConfig(accumulate_grad_batches=2, graph=graph, merge_micro_batches=False))
    # the Trainer's micro-batches run their weight gradients queued and batched (the batched split plan); the
    # plain-autograd reference takes the same plan, so the gradients stay bitwise comparable
    from matcha import _native as N

    N.lib().mtts_wgrad_plan_mode(1)
    try:
        _accumulate2_steps(tr, m_tr, m_ref, b1, b2, graph)
    finally:
        N.lib().mtts_wgrad_plan_mode(0)


@pytest.mark.parametrize("graph", [False, True])
def test_accumulate_merged_micro_batches_vs_torch(graph):
    """TrainConfig.merge_micro_batches (the default): two micro-batches of one padded shape run as ONE forward /
    backward with the losses normalised per micro-batch (MatchaTTS.forward(segments=2)).  Same mathematics as the
    reference's accumulation; the per-utterance forward is unchanged and only the weight-gradient reductions
    (over 8 utterances at once instead of 4 + 4) round differently: logged losses within 1e-6, parameters after
    1 and 3 steps within 1e-6 relative, except pure-noise gradients (Adam moves them by up to ~lr per step)."""
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    b1 = synthetic_batch(4, 24, 96, seed=1, device=DEV)
    b2 = synthetic_batch(4, 24, 96, seed=2, device=DEV)
    m_tr, m_ref = _model(7), _model(7)
    m_ref.load_state_dict(m_tr.state_dict())
    m_tr.eval()
    m_ref.eval()
    t = torch.rand(4, 1, 1, device=DEV)
    z = torch.randn(4, 80, 96, device=DEV)
    _inject(m_tr, torch.cat([t, t]), torch.cat([z, z]))  # the merged batch: both micro-batches' t / z
    _inject(m_ref, t, z)
    tr = Trainer(m_tr, TrainConfig(accumulate_grad_batches=2, graph=graph))
    assert tr._merge_ok([b1, b2])
    params = [p for p in m_ref.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-6)
    for step in range(3):
        logged = tr.step([b1, b2]).clone()
        tot = []
        for b in (b1, b2):
            dur, prior, diff, _ = m_ref(**b)
            tot.append((dur + prior + diff).detach())
            ((dur + prior + diff) / 2).backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        torch.testing.assert_close(logged[3], (tot[0] + tot[1]) / 2, rtol=2e-6, atol=0.0)
        worst = []
        for (n, a), (_, r) in zip(m_tr.named_parameters(), m_ref.named_parameters()):
            d = (a.detach() - r.detach()).abs()
            ok = d <= 1e-6 * r.detach().abs() + 1e-9
            worst.append((d.max().item(), n, int((~ok).sum())))
            assert ok.all() or d.max().item() <= (step + 1) * 2e-4 * 1.01, (step, n, d.max().item())
        print("merged", "graph" if graph else "eager", "step", step, "largest parameter differences:", sorted(worst)[-3:])


def _accumulate2_steps(tr, m_tr, m_ref, b1, b2, graph):
    params = [p for p in m_ref.parameters() if p.requires_grad]
    opt = torch.optim.AdamW(params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-6)
    for step in range(3):
        logged = tr.step([b1, b2]).clone()
        tot = []
        for b in (b1, b2):
            dur, prior, diff, _ = m_ref(**b)
            tot.append((dur + prior + diff).detach())
            ((dur + prior + diff) / 2).backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        # after the first step graph mode's parameters are ulps apart (HIP clip + AdamW), which moves the
        # losses by a few ulp of their own; eager mode stays bitwise
        rtol = 0.0 if step == 0 else (5e-6 if graph else 1e-6)
        torch.testing.assert_close(logged[3], (tot[0] + tot[1]) / 2, rtol=rtol, atol=0.0)
        if step not in (0, 2):
            continue
        worst = []
        for (n, a), (_, r) in zip(m_tr.named_parameters(), m_ref.named_parameters()):
            d = (a.detach() - r.detach()).abs()
            if not graph:  # the eager Trainer runs the reference's own optimizer: bitwise
                assert torch.equal(a.detach(), r.detach()), (step, n, d.max().item())
            elif step == 0:
                assert (d <= _ulp2(r.detach())).all(), (n, d.max().item())
            else:
                ok = d <= 1e-6 * r.detach().abs() + 1e-9
                worst.append((d.max().item(), n, int((~ok).sum())))
                assert ok.all() or d.max().item() <= 3 * 1e-4 * 1.01, (n, d.max().item())
        if worst:
            print("graph" if graph else "eager", "after 3 steps, largest parameter differences:", sorted(worst)[-4:])


def _ulp2(r):
    """2 ulp of the parameter, or -- where the parameter is smaller than the updates it has received
    (three steps of ~lr = 1e-4 each) -- 2 ulp of that accumulated update."""
    return 2 * torch.finfo(torch.float32).eps * r.abs().clamp_min(4e-4)


@pytest.mark.parametrize("graph", [False, True])
def test_decoder_prefetch_matches_inline(graph):
    """The decoder's weight packs and time path launched ahead on the side stream (Decoder.prefetch, from
    MatchaTTS.forward inside a Trainer step) give the same step as running them in place: same kernels on
    the same inputs, so losses and every parameter after one step are bitwise equal.  t / z are passed in
    the batch (the Trainer hands them to MatchaTTS.forward, which prefetches for that t)."""
    import matcha.models.matcha_tts as MT
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    b = synthetic_batch(4, 20, 80, device=DEV)
    b = dict(b, t=torch.rand(4, 1, 1, device=DEV), z=torch.randn(4, 80, 80, device=DEV))
    res = []
    saved = MT._PREFETCH
    try:
        for pf in (True, False):
            MT._PREFETCH = pf
            m = _model(5)
            m.eval()  # dropout off
            tr = Trainer(m, TrainConfig(graph=graph))
            logged = tr.step([b]).clone()
            tr.step([b])
            torch.cuda.synchronize()
            res.append((logged, {n: p.detach().clone() for n, p in m.named_parameters()}))
    finally:
        MT._PREFETCH = saved
    assert torch.equal(res[0][0], res[1][0]), (res[0][0], res[1][0])
    for n in res[0][1]:
        assert torch.equal(res[0][1][n], res[1][1][n]), n


@pytest.mark.parametrize("precision", ["32-true", "bf16-parity"])
def test_graph_gradients_equal_eager_over_replays(precision):
    """Every side-stream fork of the step (decoder prefetch of packs + time path, the seam flush of the
    decoder's queued weight gradients, the encoder's chunked side flushes, the time-MLP and embedding
    backwards on the side stream) inside the CAPTURED step: the fwd+bwd graph replayed several times gives
    gradients bitwise equal to the eager fwd+bwd, every replay.  A side-stream tensor freed and reused
    while another stream still reads it (the capture-only NaN of round 3) shows up
    here as a replay whose gradients differ."""
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    b = synthetic_batch(4, 24, 96, seed=4, device=DEV)
    b = dict(b, t=torch.rand(4, 1, 1, device=DEV), z=torch.randn(4, 80, 96, device=DEV))
    m = _model(11)
    m.eval()  # dropout off: eager and replayed steps compute the same gradients
    te = Trainer(m, TrainConfig(precision=precision, graph=False))
    for p in m.parameters():
        p.grad = None
    le = te._fwd_bwd([b]).clone()
    torch.cuda.synchronize()
    ge = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    for p in m.parameters():
        p.grad = None
    tg = Trainer(m, TrainConfig(precision=precision, graph=True))
    e = tg._graph_capture([b])
    assert len(ge) > 100
    for rep in range(4):
        e["g_fb"].replay()
        torch.cuda.synchronize()
        assert torch.equal(e["logged"], le), (rep, e["logged"], le)
        for n, p in m.named_parameters():
            if n in ge:
                assert p.grad is not None and torch.equal(p.grad, ge[n]), (rep, n)
