"""Monotonic Alignment Search on the GPU (drop-in for matcha/utils/monotonic_align/__init__.py).

Reference: /root/reference/matcha/utils/monotonic_align/__init__.py:40-55 copies the lattice to the
host, runs the Cython Viterbi (core.pyx:16-128) on CPU threads and copies the path back -- a
device->host->device round trip and a stream synchronisation in the middle of every forward pass.
Here the whole thing stays on the stream: ``mtts_maximum_path_f32`` (csrc/mas.hip) reads the fp32
lattice and mask in HBM and writes the dense path; nothing synchronises with the host.

Parity: bit-identical paths to the compiled Cython for 1 <= t_x <= t_y (the reference's pure-Python
fallback, __init__.py:8-37, uses the opposite tie rule and is NOT the parity target).
"""
from __future__ import annotations

import torch

from matcha import _native as N


def _workspace(B: int, Tx: int, Ty: int, device) -> torch.Tensor:
    nbytes = int(N.lib().mtts_maximum_path_workspace_size(B, Tx, Ty))
    return torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)


def maximum_path(value: torch.Tensor, mask: torch.Tensor, *, return_row_start: bool = False):
    """value, mask: [b, t_x, t_y]  ->  path [b, t_x, t_y] in value's dtype, on value's device.

    Same contract as the reference (__init__.py:40-55): the DP runs on value*mask in fp32,
    t_x = mask.sum(1)[:, 0], t_y = mask.sum(2)[:, 0]; the caller's tensors are not modified.
    With ``return_row_start`` also returns int32 [b, t_x] first-column-per-row (-1 = no path) and
    int32 [b, 2] lengths, which consumers (durations, mu_y gather) use instead of the dense path.
    """
    N.require_device(value, mask)
    if value.dim() != 3 or mask.shape != value.shape:
        raise ValueError(f"maximum_path expects value and mask of the same [b, t_x, t_y] shape, "
                         f"got {tuple(value.shape)} and {tuple(mask.shape)}")
    out_dtype = value.dtype
    flags = 0
    if value.dtype != torch.float32:
        # reference: value*mask in torch's promoted dtype, then .astype(np.float32) (__init__.py:45,48)
        value = (value * mask).to(torch.float32)
        flags |= N.MTTS_MAS_VALUE_PREMASKED
    if mask.dtype != torch.float32:
        mask = mask.to(torch.float32)
    value = value.contiguous()
    mask = mask.contiguous()
    B, Tx, Ty = value.shape
    dev = value.device
    path = torch.empty((B, Tx, Ty), dtype=torch.float32, device=dev)
    row_start = torch.empty((B, Tx), dtype=torch.int32, device=dev) if return_row_start else None
    lengths = torch.empty((B, 2), dtype=torch.int32, device=dev) if return_row_start else None
    ws = _workspace(B, Tx, Ty, dev)
    with torch.cuda.device(dev):
        rc = N.lib().mtts_maximum_path_f32(
            N.ptr(value), N.ptr(mask), N.ptr(path), B, Tx, Ty, flags, N.ptr(lengths),
            N.ptr(row_start), N.ptr(ws), ws.numel(), N.stream_handle(dev))
    N.check(rc, "mtts_maximum_path_f32")
    if out_dtype != torch.float32:
        path = path.to(out_dtype)
    if return_row_start:
        return path, row_start, lengths
    return path


def maximum_path_c(paths: torch.Tensor, values: torch.Tensor, t_xs: torch.Tensor,
                   t_ys: torch.Tensor, max_neg_val: float = -1e9) -> None:
    """Device twin of core.compute_batch_alignments (core.pyx:101-128), bound as maximum_path_c.

    paths int32 [b,t_x,t_y] (ones are set on the path, other entries untouched), values float32
    [b,t_x,t_y] (mutated in place to the DP lattice exactly like the Cython), t_xs/t_ys int32 [b].
    """
    N.require_device(paths, values, t_xs, t_ys)
    if paths.dtype != torch.int32 or values.dtype != torch.float32:
        raise TypeError("maximum_path_c expects int32 paths and float32 values (as the Cython)")
    if not (paths.is_contiguous() and values.is_contiguous()):
        raise ValueError("maximum_path_c mutates its arguments in place: they must be C-contiguous")
    B, Tx, Ty = values.shape
    t_xs = t_xs.to(torch.int32).contiguous()
    t_ys = t_ys.to(torch.int32).contiguous()
    dev = values.device
    ws = _workspace(B, Tx, Ty, dev)
    with torch.cuda.device(dev):
        rc = N.lib().mtts_compute_batch_alignments(
            N.ptr(paths), N.ptr(values), N.ptr(t_xs), N.ptr(t_ys), B, Tx, Ty, float(max_neg_val),
            N.ptr(ws), ws.numel(), N.stream_handle(dev))
    N.check(rc, "mtts_compute_batch_alignments")


# the reference binds the compiled core as maximum_path_c (__init__.py:4-5)
compute_batch_alignments = maximum_path_c
