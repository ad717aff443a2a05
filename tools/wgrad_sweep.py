"""Times conv_wgrad schedules (rows per step x split target) on the train step's weight-gradient shapes,
checking each result against torch first.  One JSON line per (shape, schedule)."""
import json, sys, math
from pathlib import Path
import torch
import torch.nn.functional as F
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd")]
from matcha.models.components import _ops as O

dev = torch.device("cuda")
def t_ev(fn, iters=20):
    """GPU time per call: `iters` calls captured in one HIP graph, replayed, timed with events (no
    host launch gaps in the measurement)."""
    for _ in range(3): fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters): fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3): g.replay()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / (3 * iters) * 1e3

prec_name = sys.argv[1] if len(sys.argv) > 1 else "bf16"
prec = O.PREC_BF16 if prec_name == "bf16" else O.PREC_FP32
scheds = [(32, -1, 1), (32, -1, 2), (64, -1, 1), (64, -1, 2), (32, 512, 1), (32, 512, 2), (64, 512, 2),
          (32, 1024, 1), (32, 1024, 2), (32, 128, 2), (64, 256, 2), (32, 64, 1), (32, 128, 1),
          (32, 192, 1)] if prec_name == "bf16" else [(32, -1, 1), (32, 512, 1)]
shapes = [("conv3_full_256", 32, 600, 256, 256, 3), ("conv3_half_256", 32, 300, 256, 256, 3),
          ("conv3_full_512", 32, 600, 512, 256, 3), ("lin_full_256_1024", 32, 600, 256, 1024, 1),
          ("lin_full_1024_256", 32, 600, 1024, 256, 1), ("lin_full_256_768", 32, 600, 256, 768, 1),
          ("enc_conv3_192_768", 32, 120, 192, 768, 3), ("enc_conv3_768_192", 32, 120, 768, 192, 3),
          ("enc_lin_192_576", 32, 120, 192, 576, 1), ("enc_lin_192_192", 32, 120, 192, 192, 1),
          ("half_lin_256_1024", 32, 300, 256, 1024, 1), ("half_lin_1024_256", 32, 300, 1024, 256, 1)]
if len(sys.argv) > 2:
    shapes = [s_ for s_ in shapes if s_[0] in sys.argv[2].split(",")]
for name, B, T, Cin, Cout, k in shapes:
    x = torch.randn(B, T, Cin, device=dev)
    dy = torch.randn(B, T, Cout, device=dev)
    pad = k // 2
    ref = torch.nn.grad.conv1d_weight(x.transpose(1, 2), (Cout, Cin, k), dy.transpose(1, 2), padding=pad)
    refb = dy.sum((0, 1))
    dw = torch.empty(Cout, Cin, k, device=dev)
    db = torch.empty(Cout, device=dev)
    flops = 2.0 * B * T * Cout * Cin * k
    for kb, tb, dp in scheds:
        run = lambda: O._wgrad(dy, T, 1, 0, x, T, T, B, 1, [j - pad for j in range(k)], Cin, Cout, dw, (Cin * k, k, 1),
                               prec=prec, db=db, rows_per_step=kb, target_blocks=tb, depth=dp)
        run(); torch.cuda.synchronize()
        err = ((dw - ref).norm() / ref.norm()).item()
        errb = ((db - refb).norm() / refb.norm()).item()
        us = t_ev(run)
        print(json.dumps({"shape": name, "kb": kb, "target": tb, "depth": dp, "us": round(us, 1), "tflops": round(flops / us / 1e6, 1),
                          "rel_err": float(f"{err:.2e}"), "db_err": float(f"{errb:.2e}")}), flush=True)
