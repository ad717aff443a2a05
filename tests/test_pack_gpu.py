"""Weight packing (csrc/pack.hip mtts_pack_weights) against the layouts written out in torch: every
PackSpec kind of _ops.py (linear / stacked linear and their transposes, conv, conv dgrad per stride
phase, transposed conv per output phase and its dgrad), fp32 / bf16 / split bf16 planes.  The shapes
reach both code paths: the row-gather groups and the LDS-transposed tiles of the transposing jobs
(sc > sr with C % 8 == 0), ragged tiles included.  Bit-exact."""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _pad(t, Kp):
    return F.pad(t, (0, Kp - t.shape[1]))


def _cases():
    from matcha.models.components import _ops as O

    g = torch.Generator().manual_seed(3)
    r = lambda *s: torch.randn(*s, generator=g).to(DEV)
    lin, lin2 = r(96, 40), (r(256, 192), r(64, 192), r(8, 192))
    lin1 = r(1, 192)  # N = 1: the transpose is not tileable (C % 8 != 0)
    conv, conv_odd = r(192, 80, 3), r(100, 37, 5)
    convT = r(256, 128, 4)
    cases = [
        (O.spec_linear((lin,)), lin),
        (O.spec_linear((lin,), dgrad=True), lin.T),
        (O.spec_linear(lin2), torch.cat(lin2)),
        (O.spec_linear(lin2, dgrad=True), torch.cat(lin2).T),
        (O.spec_linear((lin1,), dgrad=True), lin1.T),
        (O.spec_conv_fwd(conv), conv.permute(0, 2, 1).reshape(192, -1)),
        (O.spec_conv_fwd(conv_odd), conv_odd.permute(0, 2, 1).reshape(100, -1)),
        (O.spec_conv_dgrad(conv), conv.permute(1, 2, 0).reshape(80, -1)),
        (O.spec_conv_dgrad(conv_odd), conv_odd.permute(1, 2, 0).reshape(37, -1)),
        (O.spec_conv_dgrad(conv, 1, 2), conv[:, :, 1::2].permute(1, 2, 0).reshape(80, -1)),
        (O.spec_convT_fwd(convT, 0, 2), convT[:, :, 0::2].permute(1, 2, 0).reshape(128, -1)),
        (O.spec_convT_fwd(convT, 1, 2), convT[:, :, 1::2].permute(1, 2, 0).reshape(128, -1)),
        (O.spec_convT_dgrad(convT), convT.permute(0, 2, 1).reshape(256, -1)),
    ]
    return [(sp, _pad(ref.contiguous(), sp.Kp)) for sp, ref in cases]


@pytest.mark.parametrize("kind", ["fp32", "bf16", "split"])
def test_pack_layouts(kind):
    from matcha.models.components import _ops as O

    prec = {"fp32": O.PREC_FP32, "bf16": O.PREC_BF16, "split": O.PACK_BF16_SPLIT}[kind]
    cases = _cases()
    outs = O._run_pack([sp for sp, _ in cases], prec)  # one batched launch over every job
    torch.cuda.synchronize()
    for i, ((sp, ref), out) in enumerate(zip(cases, outs)):
        if kind == "fp32":
            assert torch.equal(out, ref), (i, sp.key[0])
        elif kind == "bf16":
            assert torch.equal(out, ref.bfloat16()), (i, sp.key[0])
        else:
            hi = ref.bfloat16()
            assert torch.equal(out[:sp.rows], hi), (i, sp.key[0])
            assert torch.equal(out[sp.rows:], (ref - hi.float()).bfloat16()), (i, sp.key[0])
