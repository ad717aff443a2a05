"""Lists the torch (non-libmtts) kernels of one eager bf16 train step by python call site: aten op, input
shapes, count, device time.  python tools/torch_glue.py [graph: 0/1]"""
import collections
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
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
    tr.step([b])
    torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0.0, 0])
for e in prof.events():
    if e.device_type.name != "CPU" or not e.kernels:
        continue
    names = [k.name for k in e.kernels]
    if any(("mtts" in n or "(anonymous namespace)::" in n) and "at::native" not in n for n in names):
        continue  # libmtts kernels
    if e.name.startswith("autograd::") or e.name in ("_ConvTMBackward",):
        pass
    site = None
    p = e
    chain = []
    while p is not None:
        if site is None and p.stack:
            fr = [s for s in p.stack if "/repo/" in s and "tools/" not in s]
            if fr:
                site = fr[0].split("/repo/")[-1]
        chain.append(p.name)
        p = p.cpu_parent
    bw = next((c for c in chain if "Backward" in c), "")
    key = f"{e.name} {str(e.input_shapes)[:70]} | {bw[:40]} | {site}"
    agg[key][0] += sum(k.duration for k in e.kernels)
    agg[key][1] += len(e.kernels)
tot = sum(v[0] for v in agg.values())
print(f"torch kernels: {sum(v[1] for v in agg.values())} launches, {tot / 1e3:.3f} ms")
for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:70]:
    print(f"{t:8.1f} us {n:4d}x  {k}")
