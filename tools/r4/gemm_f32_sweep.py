"""Schedule sweep of the parity policy's exact-fp32 text-encoder forward GEMMs (round 4): one bf16-parity
fwd+bwd of the bench batch records every O._gemm call whose packed weight is fp32 (precise_forward("fp32"));
each distinct call is re-run with every fp32 register config (0..7) x split-K count, graph-timed, its output
checked against the default schedule's.  One JSON line per call class.  python tools/r4/gemm_f32_sweep.py"""
import json
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT), str(ROOT / "tools")]
from preln_shapes import t_ev  # noqa: E402
from matcha.models.components import _ops as O  # noqa: E402
from matcha.models.matcha_tts import MatchaTTS  # noqa: E402
from matcha.training import TrainConfig, Trainer, synthetic_batch  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(1234)
model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev).train()
tr = Trainer(model, TrainConfig(precision="bf16-parity", graph=False))
batch = synthetic_batch(32, 120, 600, seed=1000, device=dev)
for _ in range(2):
    tr._fwd_bwd([batch])
torch.cuda.synchronize()

calls = {}
orig = O._gemm


def spy(A, Ti, To, nb, in_stride, offs, cin, Wp, Kp, N_, C, To_full, *a, **kw):
    out = orig(A, Ti, To, nb, in_stride, offs, cin, Wp, Kp, N_, C, To_full, *a, **kw)
    if Wp.dtype == torch.float32:
        flags = tuple(kw.get(k) is not None for k in ("a_scale", "bias", "residual", "c_scale", "C_pre", "aux"))
        key = (nb * To, N_, len(offs) * cin, cin, len(offs), kw.get("act", 0), kw.get("dropout_p", 0.0) > 0, flags)
        if key in calls:
            calls[key][0] += 1
        else:
            kw2 = dict(kw)
            for k in ("residual", "aux", "a_scale", "bias", "c_scale"):
                if kw2.get(k) is not None:
                    kw2[k] = kw2[k].clone()
            calls[key] = [1, (A.clone(), Ti, To, nb, in_stride, list(offs), cin, Wp, Kp, N_, torch.empty_like(C),
                              To_full) + tuple(a), kw2]
    return out


O._gemm = spy
tr._fwd_bwd([batch])
torch.cuda.synchronize()
O._gemm = orig
spl = [int(v) for v in os.environ.get("SWEEP_SPLITS", "1,2,3,4,6,8,12").split(",")]
total_default = total_best = 0.0
for key, (count, args, kw) in sorted(calls.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2] * kv[1][0]):
    C = args[10]

    def run(cfg, splits):
        kw2 = dict(kw, tile_cfg=cfg, splits=splits)
        return lambda: orig(*args, **kw2)

    run(-1, 0)()
    torch.cuda.synchronize()
    ref = C.float().clone()
    res = {}
    for cfg, s in [(-1, 0)] + [(c, s) for c in range(8) for s in spl]:
        fn = run(cfg, s)
        try:
            fn()
            torch.cuda.synchronize()
        except Exception:
            continue
        err = ((C.float() - ref).norm() / ref.norm().clamp_min(1e-30)).item()
        if not err < 1e-5:
            continue
        res[f"{cfg}/{s}"] = round(t_ev(fn), 1)
    best = sorted(res.items(), key=lambda kv: kv[1])[:6]
    total_default += count * res.get("-1/0", 0)
    total_best += count * best[0][1]
    print(json.dumps({"M": key[0], "N": key[1], "K": key[2], "cin": key[3], "taps": key[4], "act": key[5],
                      "drop": key[6], "flags": key[7], "count": count, "default_us": res.get("-1/0"), "best": best,
                      "gain_us_total": round(count * (res.get("-1/0", 0) - best[0][1]), 1)}), flush=True)
print(json.dumps({"total_default_us": round(total_default, 1), "total_best_us": round(total_best, 1)}))
