"""Per-launch table of the train step's conv/linear GEMMs (one eager bf16 fwd+bwd of the bench batch,
HIP events on the launch stream): python tools/step_gemms.py [cfg_override]."""
import collections
import json
import sys
from pathlib import Path
import torch
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT)]
from matcha.models.components import _ops as O
from matcha.models.matcha_tts import MatchaTTS
from matcha.training import TrainConfig, Trainer, synthetic_batch

dev = torch.device("cuda")
torch.manual_seed(1234)
model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev).train()
tr = Trainer(model, TrainConfig(precision="bf16-mixed", graph=False))
batch = synthetic_batch(32, 120, 600, seed=1000, device=dev)
for _ in range(3):
    tr._fwd_bwd([batch])
torch.cuda.synchronize()
O.LAUNCH_LOG = []
tr._fwd_bwd([batch])
torch.cuda.synchronize()
log, O.LAUNCH_LOG = O.LAUNCH_LOG, None
rows = []
for r in log:
    us = r[0].elapsed_time(r[1]) * 1e3
    d = r[5]
    rows.append((us, r[2], r[4], d))
tot = sum(x[0] for x in rows)
print(f"total {tot:.0f} us over {len(rows)} launches; {sum(x[1] for x in rows)/tot/1e6:.0f} TFLOP/s, "
      f"{sum(x[2] for x in rows)/tot/1e3:.0f} GB/s algorithmic")
agg = collections.defaultdict(lambda: [0.0, 0, 0.0, 0.0])
for us, fl, nb, d in rows:
    key = (d["M"], d["N"], d["K"], d["cin"], d["ntaps"], d["in_stride"], d["res"], d["act"], d["pre"], d["drop"], d["cs"], d["asc"], d.get("cfg", -1))
    a = agg[key]; a[0] += us; a[1] += 1; a[2] += fl; a[3] += nb
print("   us  n   avg   TF/s  GB/s   M      N    K   cin tap s res act pre drop cs asc cfg")
for k, a in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"{a[0]:6.0f} {a[1]:2d} {a[0]/a[1]:6.1f} {a[2]/a[0]/1e6:5.0f} {a[3]/a[0]/1e3:5.0f}  " + " ".join(str(int(x)) for x in k))
