"""Per-kernel floor of a graph-replayed chain on this box: 400 dependent launches of (a) a tiny torch
elementwise kernel, (b) the library's dropout kernel on one row, (c) a 3840 x 192 LayerNorm (the
encoder's shape), (d) the same LN with a 2 KiB kernel-argument struct (reduce_partials on 1 job).
Prints us per launch.  python tools/r3/launch_floor.py"""
import ctypes
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT)]
from matcha import _native as N  # noqa: E402
from matcha.models.components import _ops as O  # noqa: E402

dev = torch.device("cuda")
lib = N.lib()


def per_launch(fn, n=400):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (5 * n) * 1e3


x = torch.zeros(1, device=dev)
print("torch add_ on 1 element     %.2f us" % per_launch(lambda: x.add_(1)))
xs = torch.randn(1, 64, device=dev)
ys = torch.empty_like(xs)
seed = torch.tensor([1, 2], dtype=torch.int32, device=dev)


def drop():
    N.check(lib.mtts_dropout_apply(N.ptr(xs), N.ptr(ys), 1, 64, 64, ctypes.c_float(0.1), N.ptr(seed),
                                   torch.cuda.current_stream().cuda_stream), "drop")


try:
    print("mtts dropout on 1 row       %.2f us" % per_launch(drop))
except Exception as e:  # noqa: BLE001
    print("dropout probe failed:", e)
h = torch.randn(32, 120, 192, device=dev)
w = torch.ones(192, device=dev)
b = torch.zeros(192, device=dev)
try:
    print("encoder LayerNorm 3840x192  %.2f us" % per_launch(lambda: O.layer_norm_tm(h, w, b, 1e-5)
                                                            if hasattr(O, "layer_norm_tm") else torch.nn.functional.layer_norm(h, (192,), w, b)))
except Exception as e:  # noqa: BLE001
    print("LN probe failed:", e)
big = torch.randn(32, 120, 192, device=dev)
print("torch copy 3840x192 fp32    %.2f us" % per_launch(lambda: big.copy_(h)))
print("HIP_FORCE_DEV_KERNARG=", os.environ.get("HIP_FORCE_DEV_KERNARG"))
