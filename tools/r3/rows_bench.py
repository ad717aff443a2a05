#!/usr/bin/env python
"""Time MLP (csrc/time_mlp.hip) at the decoder's shapes (B=32, 160 -> 1024 -> 1024, 6 x 1024 -> 256):
forward + backward (8 launches) timed as a captured graph replayed back to back, for MTTS_ROWS_PASSES in {1, 2, 4, 6}, run back to back
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


def graph_of(dirty, passes):
    os.environ["MTTS_ROWS_PASSES"] = passes
    for p in list(mlp.parameters()) + [q for lin in projs for q in lin.parameters()]:
        p.grad = None
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(2):  # warm-up outside the capture (workspaces, packing)
            temb, tps = O.time_mlp(e, mlp.linear_1, mlp.linear_2, projs)
            torch.autograd.backward(tps, w)
    torch.cuda.current_stream().wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        if dirty:
            junk.fill_(1.0)
        temb, tps = O.time_mlp(e, mlp.linear_1, mlp.linear_2, projs)
        torch.autograd.backward(tps, w)
    return g


def replay_us(g, n=50):
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    torch.cuda.synchronize()
    s0.record()
    for _ in range(n):
        g.replay()
    s1.record()
    torch.cuda.synchronize()
    return s0.elapsed_time(s1) * 1e3 / n


gf = torch.cuda.CUDAGraph()
with torch.cuda.graph(gf):
    junk.fill_(1.0)
fill = replay_us(gf)
print(f"512 MB fill alone: {fill:.1f} us", flush=True)
def torch_graph():
    """the same forward + backward as torch ops (fp32; hipBLASLt GEMMs + elementwise), as a captured graph"""
    import torch.nn.functional as F

    for q in list(mlp.parameters()) + [q for lin in projs for q in lin.parameters()]:
        q.grad = None

    def run():
        temb = mlp(e)
        a2 = F.mish(temb)
        w_all = torch.cat([lin.weight for lin in projs])
        b_all = torch.cat([lin.bias for lin in projs])
        tps = F.linear(a2, w_all, b_all).split(256, dim=1)
        torch.autograd.backward(tps, w)

    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(2):
            run()
    torch.cuda.current_stream().wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    return g


print(f"torch ops (hipBLASLt): time MLP fwd+bwd graph replay {replay_us(torch_graph()):7.1f} us", flush=True)
for passes in ("1", "2", "4", "6"):
    for dirty in (False, True):
        t = replay_us(graph_of(dirty, passes))
        print(f"passes={passes} dirty={dirty}: time MLP fwd+bwd graph replay {t - (fill if dirty else 0):7.1f} us "
              f"(8 launches)", flush=True)
