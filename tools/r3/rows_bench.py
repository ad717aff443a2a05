#!/usr/bin/env python
"""Time MLP (csrc/time_mlp.hip) at the decoder's shapes (B=32, 160 -> 1024 -> 1024, 6 x 1024 -> 256):
forward and backward time per call with HIP events, for MTTS_ROWS_PASSES in {1, 2, 4, 6}, run back to back
(clean caches) and right after a 512 MB fill that leaves the L2s dirty (as in the train step, where the
time path's backward follows the decoder's big kernels)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT)]
import torch  # noqa: E402

from matcha.models.components import _ops as O  # noqa: E402
from matcha.models.components.decoder import TimeStepEmbeddingNet  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
mlp = TimeStepEmbeddingNet(160, 1024).to(dev)
projs = [torch.nn.Linear(1024, 256).to(dev) for _ in range(6)]
e = torch.randn(32, 160, device=dev)
w = [torch.randn(32, 256, device=dev) for _ in projs]
junk = torch.empty(128 * 1024 * 1024, device=dev)


def once(dirty):
    s0, s1, s2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    if dirty:
        junk.fill_(1.0)
    s0.record()
    temb, tps = O.time_mlp(e, mlp.linear_1, mlp.linear_2, projs)
    s1.record()
    if dirty:
        pass
    torch.autograd.backward(tps, w)
    s2.record()
    torch.cuda.synchronize()
    return s0.elapsed_time(s1) * 1e3, s1.elapsed_time(s2) * 1e3


for passes in ("1", "2", "4", "6"):
    os.environ["MTTS_ROWS_PASSES"] = passes
    for dirty in (False, True):
        for _ in range(3):
            once(dirty)
        r = [once(dirty) for _ in range(20)]
        f = sorted(x[0] for x in r)[10]
        b = sorted(x[1] for x in r)[10]
        print(f"passes={passes} dirty={dirty}: fwd {f:7.1f} us  bwd {b:7.1f} us (median of 20)", flush=True)
