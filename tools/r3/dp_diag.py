"""Which parameters differ between the world-size-1 DP graph step and the plain graph step (and between
two plain runs), after 1..3 steps.  Diagnostic for tests/test_dp_gpu.py."""
import os, socket, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "matcha-tts-etu-upmc-ensam_amd"))
import torch, torch.distributed as dist
import test_dp_gpu as T

s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
dist.init_process_group("nccl", rank=0, world_size=1, device_id=T.DEV)


def diff(a, b, tag):
    (_, la, pa), (_, lb, pb) = a, b
    bad = [(n, (pa[n] - pb[n]).abs().max().item(), (pa[n] != pb[n]).sum().item()) for n in pa if not torch.equal(pa[n], pb[n])]
    print(f"{tag}: logs equal {torch.equal(la, lb)}  params differing {len(bad)}/{len(pa)}", flush=True)
    for n, d, c in bad[:12]:
        print(f"    {n}: max {d:.3e}  count {c}", flush=True)


for steps in (1, 2, 3):
    r0 = T._run(False, "auto", steps)
    r1 = T._run(False, "auto", steps)
    diff(r0, r1, f"plain vs plain, {steps} steps")
    r2 = T._run(True, "rccl", steps)
    diff(r2, r0, f"dp(rccl) vs plain, {steps} steps")
dist.destroy_process_group()
