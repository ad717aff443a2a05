"""Sequence utilities of the training step (drop-in for matcha/utils/model.py).

Reference: /root/reference/matcha/utils/model.py -- sequence_mask :13-34, fix_len_compatibility
:37-57, generate_path :77-114, duration_loss :117-135, (de)normalize :138-221, aliases :224-229.
All device-side; no host synchronisation except fix_len_compatibility's int (as the reference).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def sequence_mask(lengths: torch.Tensor, max_length: int | None = None) -> torch.Tensor:
    """bool [B, max_length], True on valid positions (model.py:13-34)."""
    if max_length is None:
        max_length = int(lengths.max().item())
    pos = torch.arange(max_length, dtype=lengths.dtype, device=lengths.device)
    return pos.unsqueeze(0) < lengths.unsqueeze(1)


def fix_len_compatibility(length, num_downsamplings_in_unet: int = 2) -> int:
    """Round up to a multiple of 2**num_downsamplings (model.py:37-57)."""
    f = 2 ** num_downsamplings_in_unet
    if torch.is_tensor(length):
        return int(torch.ceil(length / f).item()) * f
    return -(-int(length) // f) * f


def generate_path(duration: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """Hard alignment from integer durations (model.py:77-114): [B, Tx] x [B, Tx, Ty] -> [B, Tx, Ty]."""
    B, Tx, Ty = mask.shape
    cum = torch.cumsum(duration, dim=1)
    path = sequence_mask(cum.reshape(B * Tx), Ty).to(mask.dtype).view(B, Tx, Ty)
    path = path - F.pad(path, (0, 0, 1, 0, 0, 0))[:, :-1]
    return path * mask


def duration_loss(logw: torch.Tensor, logw_: torch.Tensor, lengths: torch.Tensor) -> torch.Tensor:
    """sum((logw - logw_)^2) / sum(lengths) (model.py:117-135)."""
    return torch.sum((logw - logw_) ** 2) / torch.sum(lengths)


def _stat(v, ref: torch.Tensor):
    if isinstance(v, (float, int)):
        return v
    t = torch.as_tensor(v, dtype=ref.dtype, device=ref.device)
    return t.unsqueeze(-1)


def normalize(data: torch.Tensor, mu, std) -> torch.Tensor:
    return (data - _stat(mu, data)) / _stat(std, data)


def denormalize(data: torch.Tensor, mu, std) -> torch.Tensor:
    return data * _stat(std, data) + _stat(mu, data)


# reference names (model.py:224-229)
create_sequence_mask = sequence_mask
adjust_length_for_downsampling = fix_len_compatibility
build_alignment_path = generate_path
compute_duration_loss = duration_loss
apply_normalization = normalize
apply_denormalization = denormalize
