"""Schedule sweep on the train step's OWN weight-gradient calls: one eager bf16 fwd+bwd of the bench batch
records every O._wgrad_launch call; each distinct call is re-run with rows per step x split targets,
graph-timed INCLUDING its slab reduce (not deferred), output checked against the default schedule's.
MTTS_WGRAD_MINSTEPS (C++ side, default 4) caps the splits at M / (minsteps * rows_per_step).
python tools/r3/wgrad_step_sweep.py [max_rows]"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT), str(ROOT / "tools")]
from preln_shapes import t_ev  # noqa: E402
from matcha.models.components import _ops as O  # noqa: E402
from matcha.models.matcha_tts import MatchaTTS  # noqa: E402
from matcha.training import TrainConfig, Trainer, synthetic_batch  # noqa: E402

max_rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
dev = torch.device("cuda")
torch.manual_seed(1234)
model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev).train()
tr = Trainer(model, TrainConfig(precision="bf16-mixed", graph=False))
batch = synthetic_batch(32, 120, 600, seed=1000, device=dev)
for _ in range(2):
    tr._fwd_bwd([batch])
torch.cuda.synchronize()

calls = {}
orig = O._wgrad_launch


def spy(dY, To_full, out_stride, out_off, A, Ti, To, nb, in_stride, offs, cin, N_, dw, strides, **kw):
    out = orig(dY, To_full, out_stride, out_off, A, Ti, To, nb, in_stride, offs, cin, N_, dw, strides, **kw)
    if nb * To <= max_rows:
        key = (nb * To, N_, len(offs) * cin, cin, len(offs), in_stride, str(dY.dtype)[6:], str(A.dtype)[6:],
               kw.get("a_scale") is not None, kw.get("db") is not None)
        if key in calls:
            calls[key][0] += 1
        else:
            kw2 = dict(kw)
            for k in ("a_scale",):
                if kw2.get(k) is not None:
                    kw2[k] = kw2[k].clone()
            if kw2.get("db") is not None:
                kw2["db"] = torch.empty_like(kw2["db"])
            calls[key] = [1, (dY.clone(), To_full, out_stride, out_off, A.clone(), Ti, To, nb, in_stride, list(offs),
                              cin, N_, torch.empty_like(dw), strides), kw2]
    return out


O._wgrad_launch = spy
tr._fwd_bwd([batch])
torch.cuda.synchronize()
O._wgrad_launch = orig

for key, (count, args, kw) in sorted(calls.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2] * kv[1][0]):
    dw = args[12]

    def run(kb, tb):
        kw2 = dict(kw, rows_per_step=kb, target_blocks=tb, depth=1)
        return lambda: orig(*args, **kw2)

    run(-1, -1)()
    torch.cuda.synchronize()
    ref = dw.clone()
    res = {}
    for kb in (32, 64):
        for tb in (-1, 64, 128, 192, 256, 384, 512, 768, 1024):
            fn = run(kb, tb)
            try:
                fn()
                torch.cuda.synchronize()
            except Exception:
                continue
            err = ((dw - ref).norm() / ref.norm().clamp_min(1e-30)).item()
            if not err < 1e-2:
                res[f"{kb}/{tb}"] = f"BAD {err:.1e}"
                continue
            res[f"{kb}/{tb}"] = round(t_ev(fn), 1)
    good = {k: v for k, v in res.items() if not isinstance(v, str)}
    best = sorted(good.items(), key=lambda kv: kv[1])[:5]
    print(json.dumps({"M": key[0], "N": key[1], "K": key[2], "cin": key[3], "taps": key[4], "stride": key[5],
                      "dY": key[6], "A": key[7], "mask": key[8], "db": key[9], "count": count,
                      "default_us": good.get("-1/-1"), "best": best,
                      "gain_us_total": round(count * (good.get("-1/-1", 0) - best[0][1]), 1)}), flush=True)
