"""oracle/mel_oracle.py -- TEST INFRASTRUCTURE ONLY (the checker, never the product).

numpy restatement of the reference's log-mel feature path:
  MelSpectrogram  /root/reference/matcha/utils/audio_process.py:32-72 (reflect pad (n_fft-hop)/2,
                  periodic Hann window, center=False one-sided STFT, magnitude sqrt(re^2+im^2+1e-9),
                  mel_basis @ magnitude, log(clamp(x, 1e-5)))  -- spectral_normalize_torch :18-25
  mel basis       librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax) -- librosa is imported by the
                  reference (audio_process.py:4) but is not installed here and not vendored; its
                  published algorithm (librosa 0.10: slaney mel scale, htk=False, norm="slaney",
                  float32 weights) is restated in `librosa_mel` below.
Parity: the STFT / magnitude / projection / log chain is pinned by tests/golden/mel_golden.npz, which
tests/golden/make_mel_golden.py produced by running the reference's own MelSpectrogram with
`librosa_mel` standing in for librosa; the basis itself is parity unpinned against librosa (no
librosa in the image), only against its defining properties (tests/test_data_path.py).
Only tests/ may import this module.
"""
from __future__ import annotations

import numpy as np


def _hz_to_mel(f):
    # librosa.hz_to_mel(htk=False): linear below 1 kHz (f_sp = 200/3), log above (logstep ln(6.4)/27)
    f = np.asarray(f, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    mel = f / f_sp
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep, mel)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def librosa_mel(sr, n_fft, n_mels=128, fmin=0.0, fmax=None, htk=False, norm="slaney", dtype=np.float32):
    """librosa.filters.mel (0.10) restated: triangular filters on the slaney mel scale, each scaled
    to unit area (2 / bandwidth in Hz)."""
    assert not htk and norm == "slaney", "only the reference's configuration is restated"
    if fmax is None:
        fmax = float(sr) / 2
    weights = np.zeros((int(n_mels), int(1 + n_fft // 2)), dtype=dtype)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), int(n_mels) + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(int(n_mels)):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2: int(n_mels) + 2] - mel_f[: int(n_mels)])
    weights *= enorm[:, np.newaxis]
    return weights


def mel_spectrogram(y, n_fft=1024, num_mels=80, sampling_rate=22050, hop_size=256, win_size=1024, fmin=0,
                    fmax=8000):
    """y float32 [B, T] in [-1, 1] -> log-mel float32 [B, num_mels, F] (audio_process.py:54-72), in
    float64 internally (the check tolerance covers the reference's fp32 rounding)."""
    y = np.asarray(y, dtype=np.float64)
    pad = int((n_fft - hop_size) / 2)
    yp = np.pad(y, ((0, 0), (pad, pad)), mode="reflect")
    n = np.arange(win_size)
    win = 0.5 - 0.5 * np.cos(2 * np.pi * n / win_size)  # torch.hann_window(periodic=True)
    lpad = (n_fft - win_size) // 2
    w = np.zeros(n_fft)
    w[lpad: lpad + win_size] = win
    F = (yp.shape[1] - n_fft) // hop_size + 1
    idx = np.arange(n_fft)[None, :] + hop_size * np.arange(F)[:, None]
    frames = yp[:, idx] * w  # [B, F, n_fft]
    spec = np.fft.rfft(frames, axis=-1)  # [B, F, n_freq]
    mag = np.sqrt(spec.real ** 2 + spec.imag ** 2 + 1e-9)
    basis = librosa_mel(sampling_rate, n_fft, num_mels, fmin, fmax).astype(np.float64)
    mel = np.einsum("mk,bfk->bmf", basis, mag)
    return np.log(np.maximum(mel, 1e-5)).astype(np.float32)
