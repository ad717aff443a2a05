"""The train step's glue in HIP (csrc/losses.hip) against the torch expressions it replaces:
sequence masks (utils/model.py:13-34, text_encoder.py:300-303), the duration loss with its backward
(matcha_tts.py:287-288, utils/model.py:117-135), the loss sum + logged vector (baselightningmodule.py:121-128)."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("B,T", [(1, 1), (3, 17), (32, 120), (8, 4096)])
def test_sequence_mask_f32_and_key_bias(B, T):
    from matcha.models.components import _ops as O
    from matcha.utils.model import sequence_mask

    g = torch.Generator().manual_seed(B + T)
    lengths = torch.randint(0, T + 1, (B,), generator=g).to(DEV)
    lengths[0] = T
    m, kb = O.sequence_mask_f32(lengths, T, key_bias=True)
    want = sequence_mask(lengths, T).float()
    assert torch.equal(m, want)
    assert torch.equal(kb, (want - 1.0) * 1e4)
    assert torch.equal(O.sequence_mask_f32(lengths.int(), T), want)


@pytest.mark.parametrize("B,T", [(4, 24), (32, 120), (8, 512)])
def test_duration_loss_matches_torch(B, T):
    from matcha.models.components import _ops as O
    from matcha.utils.model import sequence_mask

    g = torch.Generator().manual_seed(B * T)
    lengths = torch.randint(1, T + 1, (B,), generator=g)
    lengths[0] = T
    x_mask = sequence_mask(lengths, T).float().unsqueeze(1).to(DEV)
    dur = (torch.randint(0, 12, (B, T), generator=g).float().to(DEV)) * x_mask[:, 0]  # zero durations included
    logw0 = torch.randn(B, 1, T, generator=g).to(DEV) * x_mask
    lengths = lengths.to(DEV)

    logw = logw0.clone().requires_grad_(True)
    loss = O.duration_loss_fused(logw, dur, lengths)
    loss.backward()
    ref_w = logw0.clone().requires_grad_(True)
    logw_ = torch.log(1e-8 + dur.unsqueeze(1)) * x_mask
    ref = torch.sum((ref_w - logw_) ** 2) / torch.sum(lengths)
    ref.backward()
    torch.testing.assert_close(loss, ref, rtol=2e-6, atol=0)  # fixed-order vs torch's tree sum
    torch.testing.assert_close(logw.grad, ref_w.grad, rtol=1e-6, atol=1e-9)


def test_loss_sum_and_gradients():
    from matcha.models.components import _ops as O

    vals = [torch.tensor(v, device=DEV, requires_grad=True) for v in (0.75, 2.5, 4.125)]
    total, logged = O.loss_sum(*vals)
    assert float(total) == (0.75 + 2.5) + 4.125
    assert logged.tolist() == [0.75, 2.5, 4.125, 7.375] and not logged.requires_grad
    (3.0 * total).backward()
    assert [float(v.grad) for v in vals] == [3.0, 3.0, 3.0]
    d, f = (torch.tensor(v, device=DEV, requires_grad=True) for v in (1.0, 2.0))
    total, logged = O.loss_sum(d, 0, f)  # prior_loss=False: the int 0 of the reference
    total.backward()
    assert logged.tolist() == [1.0, 0.0, 2.0, 3.0] and float(d.grad) == float(f.grad) == 1.0


@pytest.mark.parametrize("passes", ["1", "3"])
@pytest.mark.parametrize("B,width,dim", [(1, 256, 1024), (5, 256, 1024), (32, 256, 1024), (3, 32, 128), (7, 96, 200)])
def test_time_mlp_matches_torch(monkeypatch, B, width, dim, passes):
    """decoder.py:33-49 (Linear -> SiLU -> Linear) + each Resnet1D.mlp (Mish -> Linear) on the shared temb:
    the fused HIP path (csrc/time_mlp.hip) against the torch modules, forward and every weight / bias
    gradient, fp32; the reduction split over workgroups (one pass each) and over passes inside a
    workgroup (MTTS_ROWS_PASSES)."""
    monkeypatch.setenv("MTTS_ROWS_PASSES", passes)
    import torch.nn.functional as F

    from matcha.models.components import _ops as O
    from matcha.models.components.decoder import TimeStepEmbeddingNet

    torch.manual_seed(B)
    mlp = TimeStepEmbeddingNet(160, dim).to(DEV)
    projs = [torch.nn.Linear(dim, width).to(DEV) for _ in range(6)]
    e = torch.randn(B, 160, device=DEV) * 3
    temb, tps = O.time_mlp(e, mlp.linear_1, mlp.linear_2, projs)
    w = [torch.randn(B, width, device=DEV) for _ in projs]
    sum((tp * wi).sum() for tp, wi in zip(tps, w)).backward()
    got = [p.grad.clone() for p in list(mlp.parameters()) + [q for lin in projs for q in lin.parameters()]]
    for p in list(mlp.parameters()) + [q for lin in projs for q in lin.parameters()]:
        p.grad = None
    ref_temb = mlp(e)
    ref_tps = [lin(F.mish(ref_temb)) for lin in projs]
    sum((tp * wi).sum() for tp, wi in zip(ref_tps, w)).backward()
    want = [p.grad for p in list(mlp.parameters()) + [q for lin in projs for q in lin.parameters()]]
    torch.testing.assert_close(temb, ref_temb, rtol=2e-5, atol=2e-6)
    for a, b in zip(tps, ref_tps):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=2e-6)
        assert a.is_contiguous()
    for a, b in zip(got, want):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=2e-5 * b.abs().max().item())
    # deterministic: a second pass is bitwise identical
    temb2, tps2 = O.time_mlp(e, mlp.linear_1, mlp.linear_2, projs)
    assert torch.equal(temb, temb2) and all(torch.equal(a, b) for a, b in zip(tps, tps2))


@pytest.mark.parametrize("rows,n,ld", [(19200, 256, 256), (9600, 256, 512), (77, 5, 8), (1, 256, 256)])
def test_colsum_fixed_order(rows, n, ld):
    """mtts_colsum (the transposed conv's bias gradient): column sums of a row-strided matrix, 128-row
    partials + a fixed-order reduce: within fp32 rounding of the float64 sum, bitwise repeatable."""
    import ctypes

    from matcha import _native as N
    from matcha.models.components import _ops as O

    g = torch.Generator().manual_seed(rows + n)
    x = torch.randn(rows, ld, generator=g).to(DEV)
    lib = N.lib()
    outs = []
    for _ in range(2):
        ws = torch.empty(int(lib.mtts_colsum_workspace_size(rows, n)) // 4, device=DEV)
        out = torch.full((n,), float("nan"), device=DEV)
        N.check(lib.mtts_colsum(x.data_ptr(), rows, n, ld, out.data_ptr(), 0, ws.data_ptr(), ws.numel() * 4,
                                O._stream(x)), "mtts_colsum")
        outs.append(out)
    torch.cuda.synchronize()
    ref = x[:, :n].double().sum(0)
    assert (outs[0].double() - ref).abs().max().item() <= 1e-5 * max(1.0, ref.abs().max().item())
    assert torch.equal(outs[0], outs[1])
    assert ctypes  # (ctypes-bound entry point)
