"""Data path: log-mel features and batch assembly.

CPU: the numpy oracle (oracle/mel_oracle.py) against tests/golden/mel_golden.npz (the reference's own
MelSpectrogram run by tests/golden/make_mel_golden.py), the product's mel basis against the oracle's,
collate against the reference's semantics (ljspeech_datamodule.py:84-109), and the bucketing
sampler's invariants.  GPU: the HIP log-mel kernel (csrc/mel.hip) against the golden vectors and the
oracle; tolerance 1e-4 absolute on log-mel (fp32 STFT vs the reference's fp32 torch.stft)."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest
import torch

from oracle.mel_oracle import librosa_mel, mel_spectrogram

GOLD = np.load(Path(__file__).resolve().parent / "golden" / "mel_golden.npz")
CFG = dict(n_fft=1024, num_mels=80, sampling_rate=22050, hop_size=256, win_size=1024, fmin=0, fmax=8000)
MEL_TOL = 1e-4


def _wave(i):
    return GOLD[f"pcm_{i}"].astype(np.float32) / 32768.0


@pytest.mark.parametrize("i", [0, 1, 2])
def test_mel_oracle_matches_reference_golden(i):
    got = mel_spectrogram(_wave(i)[None], **CFG)[0]
    assert got.shape == GOLD[f"mel_{i}"].shape
    assert np.abs(got - GOLD[f"mel_{i}"]).max() < 1e-5


def test_mel_basis_properties_and_product_equality():
    from matcha.utils.audio_process import MelSpectrogram, slaney_mel_basis

    b = librosa_mel(22050, 1024, 80, 0, 8000)
    assert np.array_equal(b, GOLD["basis"])
    assert np.array_equal(slaney_mel_basis(22050, 1024, 80, 0, 8000).numpy(), b)
    # unit area in Hz of every slaney-normalised triangle (bin spacing sr / n_fft)
    area = b.sum(1) * (22050 / 1024)
    assert np.allclose(area[5:], 1.0, rtol=0.08)
    m = MelSpectrogram(**CFG)
    nz = b != 0
    for k in range(80):
        cols = np.nonzero(nz[k])[0]
        assert m.band_lo[k] == cols[0] and m.band_hi[k] == cols[-1] + 1
        assert nz[k, cols[0]: cols[-1] + 1].all()  # contiguous band


def test_mel_requires_device_tensor():
    from matcha import _native as N
    from matcha.utils.audio_process import MelSpectrogram

    with pytest.raises(N.NativeError):
        MelSpectrogram(**CFG)(torch.zeros(1, 4096))


def test_collate_matches_reference_semantics():
    from matcha.data_management.ljspeech_datamodule import collate

    g = torch.Generator().manual_seed(0)
    items = []
    for tx, ty in [(5, 17), (9, 11), (3, 30)]:
        items.append({"x": torch.randint(1, 150, (tx,), generator=g), "y": torch.randn(80, ty, generator=g),
                      "x_lengths": torch.tensor(tx), "y_lengths": torch.tensor(ty)})
    out = collate(items)
    assert out["x"].shape == (3, 9) and out["x"].dtype == torch.int64
    assert out["y"].shape == (3, 80, 30)
    assert out["x_lengths"].tolist() == [5, 9, 3] and out["y_lengths"].tolist() == [17, 11, 30]
    for b, it in enumerate(items):
        tx, ty = it["x"].numel(), it["y"].shape[1]
        assert torch.equal(out["x"][b, :tx], it["x"]) and (out["x"][b, tx:] == 0).all()
        assert torch.equal(out["y"][b, :, :ty], it["y"]) and (out["y"][b, :, ty:] == 0).all()


@pytest.mark.parametrize("world", [1, 2, 8])
def test_bucket_sampler_invariants(world):
    from matcha.data_management.ljspeech_datamodule import LengthBucketBatchSampler

    L = torch.randint(100, 900, (1037,), generator=torch.Generator().manual_seed(3))
    per_rank = [list(LengthBucketBatchSampler(L, 16, world, r, seed=5)) for r in range(world)]
    n = len(L) // (16 * world)
    assert all(len(p) == n for p in per_rank) and all(len(b) == 16 for p in per_rank for b in p)
    flat = [i for p in per_rank for b in p for i in b]
    assert len(flat) == len(set(flat)) == n * 16 * world
    # same global batch on every rank at step s: length strata dealt round-robin -> balanced max length
    for s in range(n):
        maxes = [max(L[i] for i in per_rank[r][s]) for r in range(world)]
        assert max(maxes) - min(maxes) <= 900 // 4
    # deterministic per (seed, epoch); epochs differ
    again = list(LengthBucketBatchSampler(L, 16, world, 0, seed=5))
    assert again == per_rank[0]
    s1 = LengthBucketBatchSampler(L, 16, world, 0, seed=5)
    s1.set_epoch(1)
    assert list(s1) != per_rank[0]


def test_bucketing_cuts_padding():
    from matcha.data_management.ljspeech_datamodule import LengthBucketBatchSampler

    L = torch.randint(100, 900, (2048,), generator=torch.Generator().manual_seed(4))

    def pad_ratio(bb):
        batches = list(LengthBucketBatchSampler(L, 32, 1, 0, bucket_batches=bb, seed=1))
        return sum(int(L[b].max()) * len(b) for b in batches) / sum(int(L[b].sum()) for b in batches)

    assert pad_ratio(32) < 1.1 < 1.5 < pad_ratio(0)


def test_quantized_padding_bounds_graph_shapes():
    """collate(x_quantum, y_quantum) on bucketed LJSpeech-like lengths: the padded shapes fall into a few
    classes (the graph-mode Trainer caches one captured step per shape), the extra padding is zeros and
    the padded fraction stays small.  (TrainConfig.graph_cache should cover the classes: each captured
    step keeps its own memory pool, a few GB at B=32 -- 288 GB of HBM holds dozens.)"""
    from matcha.data_management.ljspeech_datamodule import LengthBucketBatchSampler, collate

    g = torch.Generator().manual_seed(7)
    Ty = torch.randint(150, 900, (4096,), generator=g)
    Tx = (Ty // 5).clamp_min(8)
    shapes, real, padded = set(), 0, 0
    for b in LengthBucketBatchSampler(Ty, 32, 1, 0, bucket_batches=32, seed=2):
        items = [{"x": torch.ones(int(Tx[i]), dtype=torch.int64), "y": torch.ones(4, int(Ty[i])),
                  "x_lengths": Tx[i], "y_lengths": Ty[i]} for i in b]
        out = collate(items, x_quantum=16, y_quantum=64)
        assert out["x"].shape[1] % 16 == 0 and out["y"].shape[2] % 64 == 0
        assert out["x"].sum() == Tx[b].sum() and out["y"].sum() == 4 * Ty[b].sum()  # the extra padding is 0
        shapes.add((out["x"].shape[1], out["y"].shape[2]))
        real += int(Ty[b].sum())
        padded += out["y"].shape[2] * len(b)
    assert len(shapes) <= 24  # vs ~128 distinct (Tx, Ty) maxima without the quantum
    assert padded / real < 1.2


@pytest.mark.gpu
def test_mel_hip_matches_golden_and_oracle():
    from matcha.utils.audio_process import MelSpectrogram

    m = MelSpectrogram(**CFG)
    for i in range(3):
        y = torch.from_numpy(_wave(i))[None].cuda()
        got = m(y).cpu().numpy()[0]
        assert np.abs(got - GOLD[f"mel_{i}"]).max() < MEL_TOL, i
    g = torch.Generator().manual_seed(11)
    y = (0.3 * torch.randn(4, 30000, generator=g)).clamp(-1, 1)
    got = m(y.cuda()).cpu().numpy()
    ref = mel_spectrogram(y.numpy(), **CFG)
    assert got.shape == ref.shape == (4, 80, (30000 + 768 - 1024) // 256 + 1)
    assert np.abs(got - ref).max() < MEL_TOL
    # silence hits the clamp: log(1e-5) exactly where the projection is below it
    z = m(torch.zeros(1, 8192, device="cuda"))
    assert torch.allclose(z, torch.full_like(z, float(np.log(np.float32(1e-5)))))
