"""Times the fused training alignment step (mtts_prior_maximum_path: log-prior lattice + DP + runs) and
the mu_y gather backward (mtts_expand_rows_bwd) with HIP events, inputs resident in HBM.  The DP ring
depth is read from MTTS_MAS_RING at first launch.  Usage: python tools/prior_mas_bench.py [--iters N]"""
import argparse
import json
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT)]
from matcha import _native as N  # noqa: E402
from matcha.utils.monotonic_align import prior_maximum_path  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--configs", default="32x120x600,8x512x4096")
args = ap.parse_args()


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for cfg in args.configs.split(","):
    B, Tx, Ty = map(int, cfg.split("x"))
    g = torch.Generator().manual_seed(0)
    xl = (Tx * (0.7 + 0.3 * torch.rand(B, generator=g))).long().clamp(min=1); xl[0] = Tx
    yl = torch.maximum(xl, (Ty * (0.7 + 0.3 * torch.rand(B, generator=g))).long()); yl[0] = Ty
    mu = torch.randn(B, 80, Tx, generator=g).cuda()
    y = torch.randn(B, 80, Ty, generator=g).cuda()
    xl, yl = xl.cuda(), yl.cuda()
    out = prior_maximum_path(mu, y, xl, yl)
    ms = timed(lambda: prior_maximum_path(mu, y, xl, yl), args.iters)
    _, _, _, row_start, lengths = out
    dy = torch.randn(B, 80, Ty, device="cuda")
    dx = torch.empty(B, 80, Tx, device="cuda")
    st = N.stream_handle(dy.device)

    def bwd():
        N.check(N.lib().mtts_expand_rows_bwd(N.ptr(dy), N.ptr(row_start), N.ptr(lengths), B, 80, Tx, Ty, N.ptr(dx),
                                             st), "expand_rows_bwd")
    ms_bwd = timed(bwd, args.iters)
    # check: dx == per-row run sums (float64 reference of the same runs; order-independent tolerance)
    ref = torch.zeros(B, 80, Tx, dtype=torch.float64, device="cuda")
    attn = out[0].double()
    ref = torch.bmm(dy.double(), attn.transpose(1, 2))
    err = (dx.double() - ref).abs().max().item()
    print(json.dumps({"cfg": cfg, "ring": os.environ.get("MTTS_MAS_RING", "default"),
                      "prior_maximum_path_ms": round(ms, 4), "expand_rows_bwd_ms": round(ms_bwd, 4),
                      "bwd_max_abs_err": err}), flush=True)
