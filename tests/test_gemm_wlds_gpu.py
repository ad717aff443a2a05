"""Weight-resident GEMM schedule (csrc/conv_gemm_wlds.hip, schedule id MTTS_GEMM_WLDS): the decoder's k = 1..3 convs
and linears with K <= 768, W held in LDS for the whole launch and each 128-row tile's input rows staged once for
all taps.  Against a float64 implicit GEMM of the same bf16 operands (per-utterance zero padding at the taps, the
0/1 row mask on A's input rows, bias / dropout-free epilogue terms) and against the LDS-DMA schedule 41 on the whole
epilogue: not bitwise (another K order), within fp32 accumulation error; deterministic run to run; ragged row
counts, column counts that are not a multiple of the 64-column slice, both tap orders (forward -1,0,1 / dgrad
1,0,-1), the transposed conv's two-tap phases with a strided output, fp32 / bf16 A and C, one / two weight planes."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
WLDS = 64  # include/mtts_decoder.h MTTS_GEMM_WLDS


def _weights(N, K, split, g):
    from matcha.models.components import _ops as O

    w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV)
    if split:
        hi = w.bfloat16()
        Wp = torch.cat([hi, (w - hi.float()).bfloat16()]).contiguous()
        Wp._mtts_w_split = True
        return Wp, K, hi.float() + (w - hi.float()).bfloat16().float()
    Wp, Kp = O.pack_weight(w, O.PREC_BF16)
    return Wp, Kp, w.bfloat16().float()


@pytest.mark.parametrize("kind", ["c16", "c16_bias", "c32_bias", "c32_bias_res", "c32_cscale"])
@pytest.mark.parametrize("B,T,cin,N,taps,a16,split,masked,ostride", [
    (3, 301, 256, 256, [-1, 0, 1], True, True, True, 1),      # Block1D conv, split planes, ragged rows + mask
    (2, 600, 256, 256, [1, 0, -1], True, False, False, 1),    # its dgrad (descending taps)
    (4, 150, 256, 160, [-1, 0, 1], False, True, True, 1),     # fp32 A, N not a multiple of the slice
    (2, 300, 256, 512, [1, 0, -1], True, False, False, 1),    # N = 512 dgrad
    (3, 300, 256, 256, [0, -1], False, True, True, 2),        # ConvTranspose phase: 2 taps, strided output
    (2, 77, 768, 256, [0], True, False, False, 1),            # q|k|v dgrad (one tap, K = 768)
    (1, 4800, 256, 192, [-1, 0, 1], False, False, True, 1),   # one long utterance, N = 192
    (3, 333, 512, 256, [0], True, True, True, 1),             # one tap, K = 512
    (2, 100, 256, 256, [0], False, False, False, 1),          # one tap, K = 256, few blocks
])
def test_wlds_vs_float64_and_lds_dma(kind, B, T, cin, N, taps, a16, split, masked, ostride):
    from matcha.models.components import _ops as O

    g = torch.Generator(device="cpu").manual_seed(B * T + cin + N + len(taps))
    K = cin * len(taps)
    x = torch.randn(B, T, cin, generator=g).bfloat16().float()
    Wp, Kp, wq = _weights(N, K, split, g)
    kw = dict(act=O.ACT_NONE)
    msk = (torch.rand(B * T, generator=g) > 0.25).float() if masked else torch.ones(B * T)
    if masked:
        kw["a_scale"] = msk.to(DEV)
    c16 = kind.startswith("c16")
    To_full = T * ostride
    if "bias" in kind or kind == "c32_cscale":
        kw["bias"] = torch.randn(N, generator=g).to(DEV)
    if kind == "c32_bias_res":
        kw["residual"] = torch.randn(B, To_full, N, generator=g).to(DEV)
    if kind == "c32_cscale":
        kw["c_scale"] = (torch.rand(B * To_full, generator=g) > 0.2).float().to(DEV)
    A = x.to(DEV).bfloat16() if a16 else x.to(DEV)
    outs = []
    for cfg in (WLDS, WLDS, 41):
        C = torch.full((B, To_full, N), float("nan"), device=DEV, dtype=torch.bfloat16 if c16 else torch.float32)
        O._gemm(A, T, T, B, 1, taps, cin, Wp, Kp, N, C, To_full, out_stride=ostride, out_off=ostride - 1,
                prec=O.PREC_BF16, tile_cfg=cfg, **kw)
        torch.cuda.synchronize()
        outs.append(C.float())
    nan = torch.isnan(outs[0])
    assert torch.equal(nan, torch.isnan(outs[1])) and torch.equal(outs[0][~nan], outs[1][~nan])  # deterministic
    # float64 reference: implicit GEMM over the taps with per-utterance zero padding and the row mask on A
    xm = x.double() * msk.double().view(B, T, 1)
    ref = torch.zeros(B, T, N, dtype=torch.float64)
    wr = wq.double().cpu()[:, :K].reshape(N, len(taps), cin)
    for j, o in enumerate(taps):
        src = torch.zeros_like(xm)
        lo, hi_ = max(0, -o), min(T, T - o)
        src[:, lo:hi_] = xm[:, lo + o:hi_ + o]
        ref += src @ wr[:, j].T
    full = torch.full((B, To_full, N), float("nan"), dtype=torch.float64)
    rows = slice(ostride - 1, None, ostride)
    if "bias" in kind or kind == "c32_cscale":
        ref += kw["bias"].double().cpu()
    if kind == "c32_bias_res":
        ref += kw["residual"].double().cpu()[:, rows]
    if kind == "c32_cscale":
        ref *= kw["c_scale"].double().cpu().view(B, To_full, 1)[:, rows]
    full[:, rows] = ref
    got = outs[0].double().cpu()
    assert torch.equal(torch.isnan(got), torch.isnan(full))  # every output row written, nothing else
    ok = ~torch.isnan(full)
    scale = full[ok].abs().max().item()
    tol = (2 ** -7 if c16 else 2e-5) * scale
    assert (got[ok] - full[ok]).abs().max().item() <= tol
    assert (outs[0] - outs[2]).nan_to_num().abs().max().item() <= (2 ** -7 if c16 else 2e-5) * scale


def test_wlds_refuses_unsupported_shapes():
    """No silent fallback: an explicit request for a shape the kernel does not cover (K > 768, an activation, stride 2)
    fails loudly; the heuristic keeps the other schedules there."""
    from matcha import _native as N
    from matcha.models.components import _ops as O

    x = torch.randn(2, 50, 512, device=DEV)
    Wp, Kp = O.pack_weight(torch.randn(128, 3 * 512, device=DEV), O.PREC_BF16)
    y = torch.empty(2, 50, 128, device=DEV)
    with pytest.raises(N.NativeError):
        O._gemm(x, 50, 50, 2, 1, [-1, 0, 1], 512, Wp, Kp, 128, y, 50, prec=O.PREC_BF16, tile_cfg=WLDS)
    x = torch.randn(2, 50, 256, device=DEV)
    Wp, Kp = O.pack_weight(torch.randn(128, 256, device=DEV), O.PREC_BF16)
    with pytest.raises(N.NativeError):
        O._gemm(x, 50, 50, 2, 1, [0], 256, Wp, Kp, 128, y, 50, prec=O.PREC_BF16, tile_cfg=WLDS, act=O.ACT_RELU)
    x2 = torch.randn(2, 100, 256, device=DEV)  # the stride-2 Downsample conv
    Wp3, Kp3 = O.pack_weight(torch.randn(128, 3 * 256, device=DEV), O.PREC_BF16)
    with pytest.raises(N.NativeError):
        O._gemm(x2, 100, 50, 2, 2, [-1, 0, 1], 256, Wp3, Kp3, 128, y, 50, prec=O.PREC_BF16, tile_cfg=WLDS)
