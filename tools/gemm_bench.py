"""Isolated timing of the decoder GEMM kernels on the train step's shapes (HIP events), with
hipBLASLt (torch.matmul, bf16) on the same [M,K]x[K,N] as a yardstick.  One JSON line per shape."""
import json, sys, math
from pathlib import Path
import torch
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd")]
from matcha.models.components import _ops as O

dev = torch.device("cuda")
def t_ev(fn, iters=30):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us

shapes = [  # name, B, T, Cin, Cout, k  (conv) or linear when k == 0
    ("res_conv3_full", 32, 600, 256, 256, 3), ("res_conv3_half", 32, 300, 256, 256, 3),
    ("up_conv3_in512", 32, 300, 512, 256, 3), ("qkv_full", 32, 600, 256, 768, 0),
    ("ff1_full", 32, 600, 256, 1024, 0), ("ff2_full", 32, 600, 1024, 256, 0)]
prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
for name, B, T, Cin, Cout, k in shapes:
    x = torch.randn(B, T, Cin, device=dev)
    m = torch.ones(B, T, device=dev)
    kk = max(k, 1)
    w = torch.randn(Cout, Cin, kk, device=dev) / math.sqrt(Cin * kk)
    M = B * T
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(prec == "bf16")):
        if k:
            f = lambda: O.conv_tm(x, w, None, m, padding=k // 2)
        else:
            f = lambda: O.linear_tm(x, w[..., 0])
        us = t_ev(f)
    # pack-free kernel time: call the raw GEMM with a pre-packed weight
    p = O.PREC_BF16 if prec == "bf16" else O.PREC_FP32
    Wp, Kp = O.pack_weight(w.permute(0, 2, 1).reshape(Cout, kk * Cin), p)
    y = torch.empty(B, T, Cout, device=dev)
    offs = [j - kk // 2 for j in range(kk)]
    us_k = t_ev(lambda: O._gemm(x, T, T, B, 1, offs, Cin, Wp, Kp, Cout, y, T, prec=p, a_scale=m))
    flops = 2.0 * M * Cout * Cin * kk
    a16 = torch.randn(M, Cin * kk, device=dev, dtype=torch.bfloat16)
    b16 = torch.randn(Cin * kk, Cout, device=dev, dtype=torch.bfloat16)
    us_bl = t_ev(lambda: torch.matmul(a16, b16))
    print(json.dumps({"shape": name, "M": M, "K": Cin * kk, "N": Cout, "prec": prec, "op_us": round(us, 1),
                      "kernel_us": round(us_k, 1), "kernel_tflops": round(flops / us_k / 1e6, 1),
                      "hipblaslt_bf16_us": round(us_bl, 1), "hipblaslt_tflops": round(flops / us_bl / 1e6, 1),
                      "min_bytes_MB": round((M * Cin * 4 + M * Cout * 4) / 1e6, 1)}), flush=True)
