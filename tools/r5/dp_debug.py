"""Forced-DP (world 1, RCCL) graph step vs the plain graph step, step by step: which parameters' gradients /
values first differ (debugging aid for tests/test_dp_gpu.py)."""
import os
import socket
import sys
from pathlib import Path

import torch
import torch.distributed as dist

sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "matcha-tts-etu-upmc-ensam_amd"))
sys.path.insert(0, str(Path(__file__).resolve().parents[2] / "tests"))
DEV = torch.device("cuda:0")
from test_dp_gpu import _model, _inject  # noqa: E402
from matcha.training import TrainConfig, Trainer, synthetic_batch  # noqa: E402


def make(dp, env=None):
    b = synthetic_batch(4, 24, 96, seed=3, device=DEV)
    m = _model(11)
    t = torch.rand(4, 1, 1, generator=torch.Generator(device=DEV).manual_seed(1), device=DEV)
    z = torch.randn(4, 80, 96, generator=torch.Generator(device=DEV).manual_seed(2), device=DEV)
    _inject(m, t, z)
    old = Trainer.force_dp
    Trainer.force_dp = dp
    try:
        tr = Trainer(m, TrainConfig(graph=True, comm="rccl" if dp else "auto", bucket_mb=4.0))
    finally:
        Trainer.force_dp = old
    return tr, m, b


s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=DEV)
A = make(True)
B = make(False)
prev = None
for step in range(3):
    la = A[0].step([A[2]]).clone(); lb = B[0].step([B[2]]).clone()
    torch.cuda.synchronize()
    print("step", step, "logs equal", torch.equal(la, lb), flush=True)
    pa = dict(A[1].named_parameters()); pb = dict(B[1].named_parameters())
    bad_g = [n for n in pa if pa[n].grad is not None and pb[n].grad is not None and not torch.equal(pa[n].grad, pb[n].grad)]
    bad_p = [n for n in pa if not torch.equal(pa[n].detach(), pb[n].detach())]
    print("  grads differ:", len(bad_g), bad_g if step == 1 else bad_g[:8], flush=True)
    if prev is not None:
        stale = [n for n in bad_g if torch.equal(pa[n].grad, prev[n])]
        print("  of which equal to the previous step's gradient (stale):", len(stale), flush=True)
    prev = {n: pb[n].grad.clone() for n in pb if pb[n].grad is not None}
    print("  params differ:", len(bad_p), bad_p[:8], flush=True)
    for n in bad_g[:3]:
        print("   ", n, float((pa[n].grad - pb[n].grad).abs().max()), float(pb[n].grad.abs().max()), flush=True)
red = A[0].reducer
names = {id(p): n for n, p in A[1].named_parameters()}
for k, shapes in red.copied.items():
    print("bucket", k, "copied", len(shapes), "tensors,", sum(int(torch.tensor(s_).prod()) for s_ in shapes), "elements",
          flush=True)
s_, e_ = 0, 0
print("not in place:", [names[id(red.params[i])] for i in range(len(red.params))
                        if red.grad_refs[i] is not None and red.grad_refs[i].data_ptr() != red.views[i].data_ptr()][:60])
dist.destroy_process_group()
