"""Attribute the train step's GPU time to model code: torch.profiler over one eager bf16 fwd+bwd+opt
step (B=32, 120x600).  Prints the top ops by device time and, for the small elementwise kernels, the
python call sites that launch them."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT)]
import torch
from torch.profiler import profile, ProfilerActivity
from matcha.models.matcha_tts import MatchaTTS
from matcha.training import TrainConfig, Trainer, synthetic_batch

dev = torch.device("cuda")
torch.manual_seed(0)
m = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev).train()
tr = Trainer(m, TrainConfig(precision="bf16-mixed", graph=False))
b = synthetic_batch(32, 120, 600, device=dev)
for _ in range(3):
    tr.step([b])
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    tr.step([b])
    torch.cuda.synchronize()
ka = prof.key_averages()
print(ka.table(sort_by="self_device_time_total", row_limit=45, max_name_column_width=60))
# attribute every kernel to (top-level autograd node or forward call site in this repo)
from collections import defaultdict
agg = defaultdict(lambda: [0.0, 0])
for e in prof.events():
    if e.device_type.name != "CPU" or not e.kernels:
        continue
    kt = sum(k.duration for k in e.kernels)  # us
    top, site = e, None
    while top.cpu_parent is not None:
        top = top.cpu_parent
    chain = []
    p = e
    while p is not None:
        if not site and p.stack:
            fr = [s_ for s_ in p.stack if "/repo/" in s_ and "torch_prof" not in s_]
            if fr:
                site = fr[0]
        chain.append(p.name)
        p = p.cpu_parent
    bw = next((c for c in chain if "Backward" in c or "backward" in c), None)
    key = (bw or "fwd") + " | " + (site or chain[-1]) + " | " + e.name
    agg[key][0] += kt
    agg[key][1] += len(e.kernels)
tot = sum(v[0] for v in agg.values())
print(f"attributed {tot/1e3:.2f} ms")
for k_, (t_, n_) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:90]:
    print(f"{t_/1e3:7.3f} ms n={n_:4d}  {k_[:200]}")
