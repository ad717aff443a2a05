"""(schedule, split) sweep on the train step's GEMM shapes WITH their epilogues (graph-timed):
python tools/gemm_sweep2.py > log.  One JSON line per (shape, cfg, splits)."""
import json, sys, math
from pathlib import Path
import torch
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd")]
from matcha.models.components import _ops as O


def t_ev(fn, iters=20):
    """GPU time per call (us): `iters` calls captured in one HIP graph, replayed 3x, HIP events."""
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

dev = torch.device("cuda")
# name, B, T, cin, ntaps, N, act (0 none, 1 gelu+pre, 2 dgelu), drop, residual, a_scale, c_scale
SHAPES = [
    ("enc_ffn2_k3", 32, 120, 768, 3, 192, 0, 1, 1, 1, 1), ("enc_ffn1_k3", 32, 120, 192, 3, 768, 3, 1, 0, 1, 0),
    ("enc_dq_576", 32, 120, 576, 1, 192, 0, 0, 0, 0, 1), ("enc_pre_k5", 32, 120, 192, 5, 192, 0, 0, 0, 1, 0),
    ("enc_qkv", 32, 120, 192, 1, 576, 0, 0, 0, 1, 0), ("enc_lin192", 32, 120, 192, 1, 192, 0, 1, 1, 0, 1),
    ("dec_half_k3", 32, 300, 256, 3, 256, 0, 0, 0, 1, 0), ("dec_half_k3_512", 32, 300, 512, 3, 256, 0, 0, 0, 1, 0),
    ("ff1_half", 32, 300, 256, 1, 1024, 1, 1, 0, 0, 0), ("ff2d_half", 32, 300, 256, 1, 1024, 2, 1, 0, 0, 0),
    ("ff1_full", 32, 600, 256, 1, 1024, 1, 1, 0, 0, 0), ("ff2d_full", 32, 600, 256, 1, 1024, 2, 1, 0, 0, 0),
    ("dec_full_k3", 32, 600, 256, 3, 256, 0, 0, 0, 1, 0), ("ff2_full", 32, 600, 1024, 1, 256, 0, 0, 1, 0, 0),
]
cands = [(-1, 0), (7, 1), (12, 1), (41, 1), (42, 1), (38, 1), (44, 1), (45, 1), (41, 2), (42, 2), (44, 2), (42, 4),
         (44, 4)]
only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
if only:
    SHAPES = [s_ for s_ in SHAPES if s_[0] in only]
if len(sys.argv) > 1:
    cands = [tuple(int(v) for v in c.split(":")) for c in sys.argv[1].split(",")]
seed = torch.tensor([12345, 678], dtype=torch.int32, device=dev)
for name, B, T, cin, k, N, act, drop, res, asc, csc in SHAPES:
    M = B * T
    x = torch.randn(B, T, cin, device=dev)
    w = torch.randn(N, cin * k, device=dev) / math.sqrt(cin * k)
    Wp, Kp = O.pack_weight(w, O.PREC_BF16)
    bias = torch.randn(N, device=dev)
    m = (torch.rand(M, device=dev) > 0.1).float() if asc else None
    cs = (torch.rand(M, device=dev) > 0.1).float() if csc else None
    r = torch.randn(B, T, N, device=dev) if res else None
    aux = torch.randn(B, T, N, device=dev) if act == 2 else None
    pre = torch.empty(B, T, N, device=dev) if act == 1 else None
    actc = {0: 0, 1: 1, 2: 2, 3: 3}[act]
    y = torch.empty(B, T, N, device=dev)
    offs = [j - k // 2 for j in range(k)]
    ref = None
    for cfg, sp in cands:
        run = lambda: O._gemm(x, T, T, B, 1, offs, cin, Wp, Kp, N, y, T, prec=O.PREC_BF16, a_scale=m, bias=bias,
                              act=actc, residual=r, c_scale=cs, C_pre=pre, aux=aux, dropout_p=0.1 if drop else 0.0,
                              seed=seed, tile_cfg=cfg, splits=sp)
        try:
            run(); torch.cuda.synchronize()
        except Exception as e:  # schedule does not apply
            continue
        if ref is None:
            ref = y.clone()
        err = ((y - ref).norm() / ref.norm()).item()
        us = t_ev(run)
        print(json.dumps({"shape": name, "cfg": cfg, "splits": sp, "us": round(us, 1), "rel_vs_first": float(f"{err:.1e}")}),
              flush=True)
