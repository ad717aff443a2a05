"""Diagnose optimizer / accumulation parity differences (prints worst elements)."""
import math, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT), str(ROOT / "tests")]
import torch
from matcha.training import _FlatClipAdamW, TrainConfig, Trainer, synthetic_batch
from matcha.models.matcha_tts import MatchaTTS
DEV = torch.device("cuda:0")

def worst(tag, a, b, extra=()):
    d = (a - b).abs().reshape(-1)
    i = int(d.argmax())
    rel = d / b.abs().reshape(-1).clamp_min(1e-30)
    j = int(rel.argmax())
    print(f"{tag}: max abs {d[i].item():.3e} at {i} (a={a.reshape(-1)[i].item():.9e} b={b.reshape(-1)[i].item():.9e})"
          f" | max rel {rel[j].item():.3e} at {j} (a={a.reshape(-1)[j].item():.9e} b={b.reshape(-1)[j].item():.9e})",
          *[f"{n}={t.reshape(-1)[j].item():.9e}" for n, t in extra])

g = torch.Generator().manual_seed(5)
shapes = [(256, 160, 3), (256,), (1000,), (7, 5), (1,), (80, 256, 1), (3,)]
for scale in (10.0, 1e-3):
    init = [torch.randn(s, generator=g) for s in shapes]
    grads = [torch.randn(s, generator=g) * scale / math.sqrt(len(shapes)) for s in shapes]
    p_hip = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    p_ref = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    opt = _FlatClipAdamW(p_hip, torch.tensor(1e-4, device=DEV, dtype=torch.float64), 1.0)
    ref = torch.optim.AdamW(p_ref, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-6)
    for p, gr in zip(p_hip, grads):
        p.grad = gr.to(DEV).clone()
    for p, gr in zip(p_ref, grads):
        p.grad = gr.to(DEV).clone()
    opt.step()
    torch.nn.utils.clip_grad_norm_(p_ref, 1.0)
    ref.step()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(p_hip, p_ref)):
        o = opt.offsets[i]
        worst(f"scale {scale} param {i} p", a.detach(), b.detach(), [("g_ref(clipped)", b.grad)])
        worst(f"scale {scale} param {i} m", opt.exp_avg[o:o + a.numel()], ref.state[b]["exp_avg"].reshape(-1))
        worst(f"scale {scale} param {i} v", opt.exp_avg_sq[o:o + a.numel()], ref.state[b]["exp_avg_sq"].reshape(-1))

# accumulation: gradients of the Trainer's eager step vs the manual loop
def model(seed):
    torch.manual_seed(seed)
    return MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
b1 = synthetic_batch(4, 24, 96, seed=1, device=DEV)
b2 = synthetic_batch(4, 24, 96, seed=2, device=DEV)
m1, m2 = model(7), model(7)
m2.load_state_dict(m1.state_dict())
m1.eval(); m2.eval()
t = torch.rand(4, 1, 1, device=DEV); z = torch.randn(4, 80, 96, device=DEV)
for m in (m1, m2):
    m.decoder.compute_loss_and_prior = (lambda f: (lambda *a, **k: f(*a, **{**k, "t": t, "z": z})))(m.decoder.compute_loss_and_prior)
tr = Trainer(m1, TrainConfig(accumulate_grad_batches=2, graph=False))
snap = {}
real = tr.optimizer.step
def step_and_snap(*a, **k):
    snap.update({n: p.grad.clone() for n, p in m1.named_parameters() if p.grad is not None})
    return real(*a, **k)
tr.optimizer.step = step_and_snap
tr.step([b1, b2])
for b in (b1, b2):
    dur, prior, diff, _ = m2(**b)
    ((dur + prior + diff) / 2).backward()
params = [p for p in m2.parameters()]
torch.nn.utils.clip_grad_norm_(params, 1.0)
torch.cuda.synchronize()
ndiff = 0
for n, p in m2.named_parameters():
    if not torch.equal(snap[n], p.grad):
        ndiff += 1
        if ndiff < 6:
            worst("grad " + n, snap[n], p.grad)
print("params with non-identical clipped gradients:", ndiff, "of", len(snap))
