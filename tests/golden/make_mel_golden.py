"""Generates tests/golden/mel_golden.npz by running the reference's own log-mel path
(/root/reference/matcha/utils/audio_process.py, MelSpectrogram + load_and_process_audio's scaling) on
synthetic waveforms.  librosa (audio_process.py:4) is absent from the image: a stand-in module whose
filters.mel is oracle/mel_oracle.librosa_mel is installed first, so the fixture pins the reference's
STFT / magnitude / projection / log chain, not the basis (see oracle/mel_oracle.py).
Run here (needs /root/reference):  python tests/golden/make_mel_golden.py"""
from __future__ import annotations

import sys
import tempfile
import types
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
REF = Path("/root/reference")
sys.path.insert(0, str(ROOT))
from oracle.mel_oracle import librosa_mel  # noqa: E402


def main():
    lib = types.ModuleType("librosa")
    lib.filters = types.ModuleType("librosa.filters")
    lib.filters.mel = librosa_mel
    sys.modules["librosa"] = lib
    sys.modules["librosa.filters"] = lib.filters
    sys.path.insert(0, str(REF))
    from matcha.utils import audio_process as ap  # the reference module

    cfg = dict(n_fft=1024, num_mels=80, sampling_rate=22050, hop_size=256, win_size=1024, fmin=0, fmax=8000)
    proc = ap.MelSpectrogram(**cfg)
    rng = np.random.default_rng(2024)
    out = {}
    for i, n in enumerate([1024, 5000, 22050]):
        t = np.arange(n) / 22050.0
        pcm = (8000 * np.sin(2 * np.pi * (180 + 60 * i) * t) + rng.normal(0, 1500, n)).astype(np.int16)
        y = torch.FloatTensor(pcm.astype(np.float32)) / ap.MAX_WAV_VALUE  # load_and_process_audio :78
        mel = proc(y.unsqueeze(0))
        out[f"pcm_{i}"] = pcm
        out[f"mel_{i}"] = mel.squeeze(0).numpy().astype(np.float32)
    out["basis"] = proc.mel_basis.numpy()
    dst = Path(__file__).resolve().parent / "mel_golden.npz"
    np.savez_compressed(dst, **out)
    print("wrote", dst, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
