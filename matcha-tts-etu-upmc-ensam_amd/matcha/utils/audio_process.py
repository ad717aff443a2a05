"""Log-mel features (reference: matcha/utils/audio_process.py:1-81), with the post-STFT chain on the
MI355X: torch.stft (rocFFT) produces the complex spectrum in HBM, then ONE HIP kernel
(csrc/mel.hip, mtts_mel_log_fwd) forms the magnitude sqrt(re^2+im^2+1e-9), projects it on the
band-sparse slaney mel basis and applies log(clamp(., 1e-5)) -- the magnitude tensor and the matmul
output never round-trip through HBM.

Same names and argument meaning as the reference: MelSpectrogram(n_fft, num_mels, sampling_rate,
hop_size, win_size, fmin, fmax, center=False), __call__(y [B, T] float in [-1, 1]) -> [B, num_mels, F];
load_wav, load_and_process_audio, dynamic_range_compression_torch, spectral_normalize_torch,
MAX_WAV_VALUE.  Differences: __call__ takes DEVICE tensors (batched; the reference runs per utterance
on the CPU inside Dataset.__getitem__) and fails loudly without the HIP library -- there is no CPU
path.  librosa (reference :4) is not a dependency: `slaney_mel_basis` computes the same basis
(librosa.filters.mel, htk=False, norm="slaney") in float64 and stores it float32.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from matcha import _native as N

MAX_WAV_VALUE = 32768.0  # audio_process.py:9


def load_wav(full_path):
    """audio_process.py:13-15 (scipy.io.wavfile) -> (int16 samples, sampling rate)."""
    from scipy.io.wavfile import read

    sampling_rate, data = read(full_path)
    return data, sampling_rate


def dynamic_range_compression_torch(x, C=1, clip_val=1e-5):
    """audio_process.py:18-20."""
    return torch.log(torch.clamp(x, min=clip_val) * C)


def spectral_normalize_torch(magnitudes):
    """audio_process.py:23-25."""
    return dynamic_range_compression_torch(magnitudes)


def _hz_to_slaney_mel(hz: torch.Tensor) -> torch.Tensor:
    # linear below 1 kHz (200/3 Hz per mel), logarithmic above (ln 6.4 / 27 per mel)
    lin = hz * (3.0 / 200.0)
    return torch.where(hz >= 1000.0, 15.0 + torch.log(hz.clamp(min=1e-300) / 1000.0) * (27.0 / math.log(6.4)), lin)


def _slaney_mel_to_hz(mel: torch.Tensor) -> torch.Tensor:
    return torch.where(mel >= 15.0, 1000.0 * torch.exp((mel - 15.0) * (math.log(6.4) / 27.0)), mel * (200.0 / 3.0))


def slaney_mel_basis(sr: int, n_fft: int, n_mels: int, fmin: float = 0.0, fmax: float | None = None) -> torch.Tensor:
    """[n_mels, n_fft//2 + 1] float32: triangular filters between consecutive slaney-mel-spaced edge
    frequencies, each scaled by 2 / (upper edge - lower edge) in Hz (librosa.filters.mel)."""
    fmax = sr / 2.0 if fmax is None else float(fmax)
    freqs = torch.arange(n_fft // 2 + 1, dtype=torch.float64) * (sr / n_fft)
    edges = _slaney_mel_to_hz(torch.linspace(float(_hz_to_slaney_mel(torch.tensor(float(fmin), dtype=torch.float64))),
                                             float(_hz_to_slaney_mel(torch.tensor(fmax, dtype=torch.float64))),
                                             n_mels + 2, dtype=torch.float64))
    lo, ce, hi = edges[:-2, None], edges[1:-1, None], edges[2:, None]
    rise = (freqs[None] - lo) / (ce - lo)
    fall = (hi - freqs[None]) / (hi - ce)
    tri = torch.clamp(torch.minimum(rise, fall), min=0.0).to(torch.float32)  # librosa stores float32 first
    return (tri.double() * (2.0 / (hi - lo))).to(torch.float32)


class MelSpectrogram:
    """audio_process.py:32-72.  One instance per configuration; buffers move to the input's device on
    first use and stay there."""

    def __init__(self, n_fft, num_mels, sampling_rate, hop_size, win_size, fmin, fmax, center=False):
        self.n_fft = n_fft
        self.num_mels = num_mels
        self.sampling_rate = sampling_rate
        self.hop_size = hop_size
        self.win_size = win_size
        self.fmin = fmin
        self.fmax = fmax
        self.center = center
        self.mel_basis = slaney_mel_basis(sampling_rate, n_fft, num_mels, fmin, fmax)
        nz = self.mel_basis != 0
        any_nz = nz.any(1)
        first = torch.where(any_nz, nz.float().argmax(1), torch.zeros_like(any_nz, dtype=torch.long))
        last = torch.where(any_nz, nz.shape[1] - nz.flip(1).float().argmax(1), torch.zeros_like(first))
        self.band_lo = first.to(torch.int32)
        self.band_hi = last.to(torch.int32)
        self.hann_window = torch.hann_window(win_size)
        self._dev = {}

    def _buffers(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = (self.mel_basis.to(device).contiguous(), self.band_lo.to(device), self.band_hi.to(device),
                              self.hann_window.to(device))
        return self._dev[key]

    def _stft(self, y):
        pad_size = int((self.n_fft - self.hop_size) / 2)  # :47
        y = torch.nn.functional.pad(y.unsqueeze(1), (pad_size, pad_size), mode="reflect").squeeze(1)
        return torch.stft(y, self.n_fft, hop_length=self.hop_size, win_length=self.win_size,
                          window=self._buffers(y.device)[3], center=self.center, pad_mode="reflect",
                          normalized=False, onesided=True, return_complex=True)

    def _apply_stft(self, y):
        """:45-58 (magnitude spectrogram, unfused; kept for API parity)."""
        spec = self._stft(y)
        return torch.sqrt(torch.view_as_real(spec).pow(2).sum(-1) + 1e-9)

    def __call__(self, y):
        """:60-72 -> log-mel [B, num_mels, F] float32."""
        N.require_device(y)
        if y.dim() != 2:
            raise ValueError(f"MelSpectrogram expects y [B, T], got {tuple(y.shape)}")
        spec = torch.view_as_real(self._stft(y.to(torch.float32))).contiguous()  # [B, n_freq, F, 2]
        B, n_freq, F, _ = spec.shape
        basis, lo, hi, _ = self._buffers(y.device)
        out = torch.empty((B, self.num_mels, F), dtype=torch.float32, device=y.device)
        with torch.cuda.device(y.device):
            rc = N.lib().mtts_mel_log_fwd(N.ptr(spec), N.ptr(basis), N.ptr(lo), N.ptr(hi), B, n_freq, F,
                                          self.num_mels, 1e-5, N.ptr(out), N.stream_handle(y.device))
        N.check(rc, "mtts_mel_log_fwd")
        return out


def load_and_process_audio(file_path, mel_processor, device="cuda"):
    """audio_process.py:75-81: int16 wav -> float / 32768 -> [1, T] on `device` -> mel_processor."""
    sampling_rate, data = load_wav(file_path)[::-1]
    y = torch.from_numpy(np.asarray(data, dtype=np.float32)) / MAX_WAV_VALUE
    return mel_processor(y.unsqueeze(0).to(device))
