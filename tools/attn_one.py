"""Times the flash-attention kernels alone at the decoder's shapes (bf16 MFMA, fp32 I/O):
python tools/attn_one.py [T] [D] [iters] -> us per fwd / bwd call and TFLOP/s (for rocprofv3 passes)."""
import sys
from pathlib import Path
import torch
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd")]
from matcha.models.components import _ops as O

T = int(sys.argv[1]) if len(sys.argv) > 1 else 600
D = int(sys.argv[2]) if len(sys.argv) > 2 else 64
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
io16 = len(sys.argv) > 4 and sys.argv[4] == "io16"  # bf16 q|k|v / o / dO storage, as the decoder runs it
B, H = 32, 4 if D == 64 else 2
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(B, T, 3 * H * D, device=dev, generator=g, requires_grad=True)
lens = (T * (0.7 + 0.3 * torch.rand(B, device=dev, generator=g))).long()
lens[0] = T
bias = (torch.arange(T, device=dev)[None] < lens[:, None]).float()
dout = torch.randn(B, T, H * D, device=dev, generator=g)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
if io16:  # the raw entry points (no autograd), bf16 storage, timed per call under rocprofv3
    x = qkv.detach().bfloat16()
    o = torch.empty(B, T, H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, T, device=dev)
    do16 = dout.bfloat16()
    for i in range(iters + 3):
        if i == 3:
            ev[0].record()
        O._attn_fwd(x, bias, o, lse, H, O.PREC_BF16)
        if i == 3:
            ev[1].record()
            ev[2].record()
        O._attn_bwd(do16, x, bias, o, lse, H, O.PREC_BF16)
        if i == 3:
            ev[3].record()
    torch.cuda.synchronize()
    print(f"io16 T={T} D={D}: fwd {ev[0].elapsed_time(ev[1]) * 1e3:.1f} us  bwd {ev[2].elapsed_time(ev[3]) * 1e3:.1f} us")
    sys.exit(0)
with torch.autocast("cuda", dtype=torch.bfloat16):
    for i in range(iters + 3):
        if i == 3:
            ev[0].record()
        o = O.attention_tm(qkv, bias, H)
        if i == 3:
            ev[1].record()
        if i == 3:
            ev[2].record()
        (dq,) = torch.autograd.grad(o, qkv, dout)
        if i == 3:
            ev[3].record()
torch.cuda.synchronize()
f = 4.0 * B * H * T * T * D
tf, tb = ev[0].elapsed_time(ev[1]) * 1e3, ev[2].elapsed_time(ev[3]) * 1e3
print(f"T={T} D={D} B={B} H={H}: fwd {tf:.1f} us ({f / tf / 1e6:.0f} TFLOP/s)  bwd {tb:.1f} us "
      f"({2.5 * f / tb / 1e6:.0f} TFLOP/s incl. other kernels)")
