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


def _check_tx(Tx: int, limit: int | None = None) -> None:
    """The DP keeps one utterance's text rows in one workgroup's registers (8 waves x 16 rows per lane at
    most, csrc/mas.hip mas_dp_mw_kernel): t_x <= 8192 (round 6; 4096 before), and 4096 for the row-major
    lattice compute_batch_alignments mutates.  The reference Cython (core.pyx:14-96) has no cap; LJSpeech tops
    out near 190 tokens and BASELINE config 5 uses 512, so the limit is a documented shape error, not a silent
    truncation."""
    limit = N.MTTS_MAS_MAX_TX if limit is None else limit
    if Tx > limit:
        raise ValueError(f"maximum_path: text length {Tx} exceeds the GPU kernel's limit of "
                         f"{limit} rows (MTTS_MAS_MAX_TX{'' if limit == N.MTTS_MAS_MAX_TX else '_ROW_MAJOR'}, "
                         f"include/mtts.h)")


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
    _check_tx(Tx)
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
    _check_tx(Tx, N.MTTS_MAS_MAX_TX_ROW_MAJOR)
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


def prior_maximum_path(mu_x: torch.Tensor, y: torch.Tensor, x_lengths: torch.Tensor, y_lengths: torch.Tensor, *,
                       return_lattice: bool = False):
    """The training forward's alignment step fused (matcha_tts.py:276-288, MatchaTTS.forward):
    log-prior lattice from mu_x [B,C,Tx] and y [B,C,Ty] (fp32), masked by the length masks, Viterbi
    max path, and the duration target -- one lattice write to HBM instead of two bmm's, their
    elementwise tail, the [B,Tx,Ty] attention mask and a reduction over the dense path
    (csrc/mas.hip: log_prior_kernel -> mas_dp_kernel -> mas_expand_kernel / mas_runs_kernel).

    Returns (attn [B,Tx,Ty] fp32, dur [B,Tx] fp32 = attn.sum(-1), col_row [B,Ty] int32 = text row of
    each frame (-1 past t_y), row_start [B,Tx] int32, lengths [B,2] int32) and, with
    ``return_lattice``, the masked fp32 lattice [B,Tx,Ty] the DP ran on.  No gradient."""
    N.require_device(mu_x, y, x_lengths, y_lengths)
    if mu_x.dim() != 3 or y.dim() != 3 or mu_x.shape[:2] != y.shape[:2]:
        raise ValueError(f"prior_maximum_path expects mu_x [B,C,Tx] and y [B,C,Ty], got {tuple(mu_x.shape)}, "
                         f"{tuple(y.shape)}")
    mu_x = mu_x.detach().to(torch.float32).contiguous()
    y = y.detach().to(torch.float32).contiguous()
    xl = x_lengths.detach().to(torch.int64).contiguous()
    yl = y_lengths.detach().to(torch.int64).contiguous()
    B, C, Tx = mu_x.shape
    _check_tx(Tx)
    Ty = y.shape[2]
    dev = mu_x.device
    attn = torch.empty((B, Tx, Ty), dtype=torch.float32, device=dev)
    dur = torch.empty((B, Tx), dtype=torch.float32, device=dev)
    col_row = torch.empty((B, Ty), dtype=torch.int32, device=dev)
    row_start = torch.empty((B, Tx), dtype=torch.int32, device=dev)
    lengths = torch.empty((B, 2), dtype=torch.int32, device=dev)
    lattice = torch.empty((B, Tx, Ty), dtype=torch.float32, device=dev) if return_lattice else None
    ws = torch.empty(max(int(N.lib().mtts_prior_maximum_path_workspace_size(B, Tx, Ty)), 1), dtype=torch.uint8,
                     device=dev)
    with torch.cuda.device(dev):
        rc = N.lib().mtts_prior_maximum_path(
            N.ptr(mu_x), N.ptr(y), N.ptr(xl), N.ptr(yl), B, C, Tx, Ty, N.ptr(attn), N.ptr(lengths), N.ptr(row_start),
            N.ptr(dur), N.ptr(col_row), N.ptr(lattice), N.ptr(ws), ws.numel(), N.stream_handle(dev))
    N.check(rc, "mtts_prior_maximum_path")
    out = (attn, dur, col_row, row_start, lengths)
    return out + (lattice,) if return_lattice else out


class _ExpandRows(torch.autograd.Function):
    """mu_y = attn^T @ mu_x for a hard alignment (matcha_tts.py:314-315) as a gather of mu_x columns;
    backward sums each text row's run of frames (deterministic segment sums, no atomics)."""

    @staticmethod
    def forward(ctx, mu_x, col_row, row_start, lengths):
        mu_x = mu_x.to(torch.float32).contiguous()
        B, C, Tx = mu_x.shape
        Ty = col_row.shape[1]
        out = torch.empty((B, C, Ty), dtype=torch.float32, device=mu_x.device)
        N.check(N.lib().mtts_expand_rows_fwd(N.ptr(mu_x), N.ptr(col_row), B, C, Tx, Ty, N.ptr(out),
                                             N.stream_handle(mu_x.device)), "mtts_expand_rows_fwd")
        ctx.save_for_backward(row_start, lengths)
        ctx.shape = (B, C, Tx, Ty)
        return out

    @staticmethod
    def backward(ctx, dy):
        row_start, lengths = ctx.saved_tensors
        B, C, Tx, Ty = ctx.shape
        dy = dy.to(torch.float32).contiguous()
        dx = torch.empty((B, C, Tx), dtype=torch.float32, device=dy.device)
        N.check(N.lib().mtts_expand_rows_bwd(N.ptr(dy), N.ptr(row_start), N.ptr(lengths), B, C, Tx, Ty, N.ptr(dx),
                                             N.stream_handle(dy.device)), "mtts_expand_rows_bwd")
        return dx, None, None, None


def expand_rows(mu_x: torch.Tensor, col_row: torch.Tensor, row_start: torch.Tensor, lengths: torch.Tensor):
    """[B,C,Tx] -> [B,C,Ty]: attn^T @ mu_x for the alignment prior_maximum_path returned (bitwise
    equal to the bmm on the one-hot attn: every other term is 0 * finite)."""
    N.require_device(mu_x, col_row, row_start, lengths)
    return _ExpandRows.apply(mu_x, col_row, row_start, lengths)
