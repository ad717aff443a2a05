"""Every conv_gemm schedule on the train step's GEMM shapes, fp32 and bf16 A, graph-timed; one JSON
line per (shape, A storage) with all timings.  python tools/gemm_tall_sweep.py [names] > log"""
import json, math, sys
from pathlib import Path
import torch
sys.path[:0] = [str(Path(__file__).resolve().parent), str(Path(__file__).resolve().parent.parent / "matcha-tts-etu-upmc-ensam_amd")]
from preln_shapes import t_ev  # noqa: E402
from matcha.models.components import _ops as O  # noqa: E402

dev = torch.device("cuda")
P = O.PREC_BF16
seed = torch.tensor([12345, 678], dtype=torch.int32, device=dev)
# name, B, T, cin, taps, N, residual, mask, act
SHAPES = [("dec_full_k3", 32, 600, 256, 3, 256, 0, 1, 0), ("dec_half_k3", 32, 300, 256, 3, 256, 0, 1, 0),
          ("up_full_k3_512", 32, 600, 512, 3, 256, 0, 1, 0), ("ff2_full", 32, 600, 1024, 1, 256, 1, 0, 0),
          ("qkv_full", 32, 600, 256, 1, 768, 0, 0, 0), ("out_full", 32, 600, 256, 1, 256, 1, 0, 0),
          ("ff2_half", 32, 300, 1024, 1, 256, 1, 0, 0), ("enc_k3_768_192", 32, 120, 768, 3, 192, 1, 1, 0),
          ("enc_k3_192_768", 32, 120, 192, 3, 768, 0, 1, O.ACT_RELU)]
only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
for name, B, T, cin, k, N, res, msk, act in SHAPES:
    if only and name not in only:
        continue
    M = B * T
    x32 = torch.randn(B, T, cin, device=dev)
    w = torch.randn(N, cin * k, device=dev) / math.sqrt(cin * k)
    Wp, Kp = O.pack_weight(w, P)
    bias = torch.randn(N, device=dev)
    m = (torch.rand(B, T, device=dev) > 0.1).float() if msk else None
    r = torch.randn(B, T, N, device=dev) if res else None
    y = torch.empty(B, T, N, device=dev)
    offs = [j - k // 2 for j in range(k)]
    # independent fp32 reference: conv1d of the masked input (+ bias, ReLU, residual)
    xm = x32 * m.unsqueeze(-1) if m is not None else x32
    ref = torch.nn.functional.conv1d(xm.transpose(1, 2), w.view(N, k, cin).permute(0, 2, 1), bias,
                                     padding=k // 2).transpose(1, 2)
    if act == O.ACT_RELU:
        ref = ref.relu()
    if r is not None:
        ref = ref + r
    for a16 in (False, True):
        x = x32.to(torch.bfloat16) if a16 else x32
        cands = [-1] + list(range(32, 55)) + ([] if a16 else [7, 12])
        res_t = {}
        for cfg in cands:
            run = lambda: O._gemm(x, T, T, B, 1, offs, cin, Wp, Kp, N, y, T, prec=P, a_scale=m, bias=bias,
                                  residual=r, act=act, seed=seed, tile_cfg=cfg)
            try:
                run(); torch.cuda.synchronize()
            except Exception:
                continue
            err = ((y - ref).norm() / ref.norm()).item()
            if err > 1e-2:
                res_t[cfg] = f"BAD {err:.1e}"
                continue
            res_t[cfg] = round(t_ev(run), 1)
        good = {c: v for c, v in res_t.items() if not isinstance(v, str)}
        best = min(good, key=good.get)
        print(json.dumps({"shape": name, "M": M, "N": N, "K": cin * k, "A": "bf16" if a16 else "fp32",
                          "default": res_t.get(-1), "best_cfg": best, "best_us": good[best],
                          "tflops_best": round(2 * M * N * cin * k / good[best] / 1e6, 1), "all": res_t}), flush=True)
