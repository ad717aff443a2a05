"""Times every conv_gemm tile configuration on the train step's GEMM shapes (forward AND the dgrad
shapes), verifying each result against torch first.  Prints one JSON line per (shape, config)."""
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
cfgs = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else list(range(8))
prec = O.PREC_BF16 if prec_name == "bf16" else O.PREC_FP32
shapes = [("conv3_full_256", 32, 600, 256, 256, 3), ("conv3_half_256", 32, 300, 256, 256, 3),
          ("conv3_half_512", 32, 300, 512, 256, 3), ("conv3_full_512", 32, 600, 512, 256, 3),
          ("conv3_full_160", 32, 600, 160, 256, 3), ("lin_full_256_768", 32, 600, 256, 768, 1),
          ("lin_full_256_1024", 32, 600, 256, 1024, 1), ("lin_full_1024_256", 32, 600, 1024, 256, 1),
          ("lin_half_256_1024", 32, 300, 256, 1024, 1), ("lin_half_1024_256", 32, 300, 1024, 256, 1),
          ("lin_full_256_256", 32, 600, 256, 256, 1), ("lin_full_256_80", 32, 600, 256, 80, 1),
          ("down_s2_256", 32, 600, 256, 256, -3), ("lin_full_80_256", 32, 600, 80, 256, 1),
          ("conv3_full_336", 32, 600, 336, 256, 3)]

# full-epilogue equivalence of every requested config against config 7 (itself tested vs torch in
# tests/test_decoder_ops_gpu.py): mask, bias, GELU + C_pre, dropout, residual, c_scale, strided output
if prec_name == "bf16":
    B, T, Cin, Cout = 5, 77, 256, 320
    x = torch.randn(B, T, Cin, device=dev)
    msk = (torch.rand(B * T, device=dev) > 0.2).float()
    w = torch.randn(Cout, Cin * 3, device=dev) / math.sqrt(Cin * 3)
    Wp, Kp = O.pack_weight(w, prec)
    bias = torch.randn(Cout, device=dev)
    res = torch.randn(B, 2 * T, Cout, device=dev)
    cs = torch.rand(B * 2 * T, device=dev)
    seed = torch.tensor([12345, 678], dtype=torch.int32, device=dev)
    outs = {}
    for cfg in [7] + [c for c in cfgs if c != 7]:  # 64 = panel schedule
        y = torch.zeros(B, 2 * T, Cout, device=dev)
        pre = torch.zeros(B, 2 * T, Cout, device=dev)
        O._gemm(x, T, T, B, 1, [-1, 0, 1], Cin, Wp, Kp, Cout, y, 2 * T, 2, 1, prec=prec, a_scale=msk, bias=bias,
                act=1, residual=res, c_scale=cs, C_pre=pre, dropout_p=0.1, seed=seed, tile_cfg=cfg,
                binary_scale=True)
        torch.cuda.synchronize()
        outs[cfg] = (y, pre)
        e = max(((y - outs[7][0]).norm() / outs[7][0].norm()).item(), ((pre - outs[7][1]).norm() / outs[7][1].norm()).item())
        print(json.dumps({"check": "epilogue_vs_cfg7", "cfg": cfg, "rel_err": float(f"{e:.2e}"),
                          "even_rows_untouched": bool((y[:, 0::2] == 0).all().item())}), flush=True)

for name, B, T, Cin, Cout, k in shapes:
    stride = 2 if k < 0 else 1
    k = abs(k)
    To = T // stride
    x = torch.randn(B, T, Cin, device=dev)
    w = torch.randn(Cout, Cin, k, device=dev) / math.sqrt(Cin * k)
    ref = F.conv1d(x.transpose(1, 2), w, padding=k // 2, stride=stride).transpose(1, 2)
    Wp, Kp = O.pack_weight(w.permute(0, 2, 1).reshape(Cout, k * Cin), prec)
    y = torch.empty(B, To, Cout, device=dev)
    offs = [j - k // 2 for j in range(k)]
    flops = 2.0 * B * To * Cout * Cin * k
    for cfg in cfgs:
        run = lambda: O._gemm(x, T, To, B, stride, offs, Cin, Wp, Kp, Cout, y, To, prec=prec, tile_cfg=cfg)
        y.zero_(); run(); torch.cuda.synchronize()
        err = ((y - ref).norm() / ref.norm()).item()
        us = t_ev(run)
        print(json.dumps({"shape": name, "cfg": cfg, "prec": prec_name, "us": round(us, 1),
                          "tflops": round(flops / us / 1e6, 1), "rel_err": float(f"{err:.2e}")}), flush=True)
