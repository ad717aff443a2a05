"""Times the GPU log-mel path on an LJSpeech-shaped batch (B=32 utterances x 600 frames): the whole
MelSpectrogram call (reflect pad + torch.stft + the fused HIP kernel) and the HIP kernel alone (HIP
events on the launch stream), with the kernel's HBM roofline (algorithmic bytes = complex spectrum
read once, 8 B per (bin, frame), + log-mel written, 4 B per (mel, frame)).  Prints one JSON line."""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT)]
from matcha import _native as N  # noqa: E402
from matcha.utils.audio_process import MelSpectrogram  # noqa: E402

B, FR = 32, 600
T = (FR - 1) * 256 + 1024 - 768
m = MelSpectrogram(1024, 80, 22050, 256, 1024, 0, 8000)
y = (0.3 * torch.randn(B, T, generator=torch.Generator().manual_seed(0))).clamp(-1, 1).cuda()
out = m(y)
assert out.shape == (B, 80, FR), out.shape
spec = torch.view_as_real(m._stft(y)).contiguous()
basis, lo, hi, _ = m._buffers(y.device)
res = torch.empty_like(out)
st = N.stream_handle(y.device)


def kern():
    N.check(N.lib().mtts_mel_log_fwd(N.ptr(spec), N.ptr(basis), N.ptr(lo), N.ptr(hi), B, 513, FR, 80, 1e-5,
                                     N.ptr(res), st), "mel")


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


ms_call = timed(lambda: m(y))
ms_k = timed(kern)
assert torch.equal(res, out)
bytes_k = B * FR * (513 * 8 + 80 * 4)
print(json.dumps({"workload": f"log-mel B={B} x {FR} frames (n_fft 1024, hop 256, 80 mels)",
                  "ms_per_call": round(ms_call, 4), "frames_per_s": round(B * FR / ms_call * 1e3, 1),
                  "kernel_ms": round(ms_k, 4), "kernel_roofline": {"bound": "hbm", "achieved": round(bytes_k / ms_k / 1e6, 1),
                                                                   "peak": 8000.0, "unit": "GB/s",
                                                                   "frac": round(bytes_k / ms_k / 1e6 / 8000.0, 4),
                                                                   "algorithmic_bytes_per_launch": bytes_k}}))
