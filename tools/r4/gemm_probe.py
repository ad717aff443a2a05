"""Where a step GEMM's time goes: graph-timed back-to-back launches (20 per graph, the ~1.5 us kernel
boundary included) of the decoder's conv GEMM shape at growing M -- the intercept of time vs M is the fixed
cost per launch (prologue, pipeline fill, epilogue tail, boundary), the slope its streaming rate -- and at
one K step (K = 64) against the full K.  python tools/r4/gemm_probe.py [cfg ...]  (cfg: schedule ids, -1 =
the heuristic's pick)"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT), str(ROOT / "tools")]
from preln_shapes import t_ev  # noqa: E402
from matcha.models.components import _ops as O  # noqa: E402

dev = torch.device("cuda")
cfgs = [int(c) for c in sys.argv[1:]] or [-1]


def case(M, N, cin, taps, a16, c16, split=False, cfg=-1, T=600):
    nb = max(M // T, 1)
    T = M // nb
    g = torch.Generator(device="cpu").manual_seed(M + N)
    A = torch.randn(nb, T, cin, generator=g).to(dev)
    A = A.bfloat16() if a16 else A
    w = (torch.randn(N, cin, taps, generator=g) / (cin * taps) ** 0.5).to(dev)
    old = O.set_weight_split(split)
    Wp, Kp = O.packed(O.spec_conv_fwd(w), O.PREC_BF16)
    O.set_weight_split(old)
    b = torch.randn(N, generator=g).to(dev)
    m = torch.ones(nb, T, device=dev)
    C = torch.empty(nb, T, N, device=dev, dtype=torch.bfloat16 if c16 else torch.float32)
    offs = [j - taps // 2 for j in range(taps)]

    def fn():
        O._gemm(A, T, T, nb, 1, offs, cin, Wp, Kp, N, C, T, prec=O.PREC_BF16, a_scale=m, bias=b, tile_cfg=cfg)
    return t_ev(fn)


rows = []
for cfg in cfgs:
    for a16, c16 in ((True, True), (False, True)):
        for split in (False, True):
            for M in (1200, 2400, 4800, 9600, 19200, 38400):
                us = case(M, 256, 256, 3, a16, c16, split, cfg)
                one = case(M, 256, 64, 1, a16, c16, split, cfg)  # one K step
                rows.append(dict(cfg=cfg, a16=a16, c16=c16, split=split, M=M, us_k768=round(us, 2), us_k64=round(one, 2)))
                print(json.dumps(rows[-1]), flush=True)
