"""CPU restatement of the log-prior lattice and the alignment consumers -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module (the product never does).  It restates, in numpy fp32:
  * the lattice producer of MatchaTTS.forward, reference matcha/models/matcha_tts.py:277-282
        const = -0.5 * log(2 pi) * n_feats
        factor = -0.5 * ones(mu_x.shape)
        y_square = factor^T @ y**2 ;  y_mu_double = (2 * factor * mu_x)^T @ y
        mu_square = sum(factor * mu_x**2, 1)
        log_prior = y_square - y_mu_double + mu_square + const
    with the sums taken in ascending channel order, one fp32 multiply and one fp32 add per term
    (numpy float32 arithmetic is IEEE single and never contracted), which is the order
    csrc/mas.hip:log_prior_kernel uses -- so the two agree BIT FOR BIT.  The reference's torch
    matmuls sum in an implementation-defined (blocked) order; against them the lattice agrees to
    fp32 rounding, and the alignments agree exactly unless a DP decision is a near-tie.
  * maximum_path's value * mask (monotonic_align/__init__.py:45) with mask = x_mask[i] * y_mask[j]
    (matcha_tts.py:276).
  * the consumers of the hard alignment, matcha_tts.py:287-288 and 504-505:
        durations  sum_y attn[b, x, y]          (logw_ = log(1e-8 + durations) * x_mask)
        mu_y       attn^T @ mu_x               (a gather of mu_x columns on a one-hot attn)
"""
from __future__ import annotations

import math

import numpy as np


def log_prior_lattice(mu_x: np.ndarray, y: np.ndarray, x_lengths, y_lengths) -> np.ndarray:
    """mu_x [B,C,Tx], y [B,C,Ty] float32 -> masked lattice [B,Tx,Ty] float32 (premasked value)."""
    mu = np.asarray(mu_x, np.float32)
    yy = np.asarray(y, np.float32)
    B, C, Tx = mu.shape
    Ty = yy.shape[2]
    half = np.float32(-0.5)
    ysq = np.zeros((B, Ty), np.float32)
    musq = np.zeros((B, Tx), np.float32)
    ymu = np.zeros((B, Tx, Ty), np.float32)
    for c in range(C):
        m = mu[:, c, :]
        v = yy[:, c, :]
        musq = musq + half * (m * m)
        ysq = ysq + half * (v * v)
        ymu = ymu + (-m)[:, :, None] * v[:, None, :]
    cst = np.float32(-0.5 * math.log(2 * math.pi) * C)
    lat = ((ysq[:, None, :] - ymu) + musq[:, :, None]) + cst
    xl = np.clip(np.asarray(x_lengths).astype(np.int64), 0, Tx)
    yl = np.clip(np.asarray(y_lengths).astype(np.int64), 0, Ty)
    mask = ((np.arange(Tx)[None, :, None] < xl[:, None, None]) &
            (np.arange(Ty)[None, None, :] < yl[:, None, None])).astype(np.float32)
    return (lat * mask).astype(np.float32), mask


def durations(path: np.ndarray) -> np.ndarray:
    """sum_y attn[b, x, y] as float32 [B, Tx] (matcha_tts.py:287)."""
    return np.asarray(path, np.float32).sum(-1, dtype=np.float32)


def col_row(path: np.ndarray) -> np.ndarray:
    """The text row of every frame of a one-hot path [B,Tx,Ty] -> int32 [B,Ty] (-1: no row)."""
    p = np.asarray(path) != 0
    idx = p.argmax(1).astype(np.int32)
    idx[~p.any(1)] = -1
    return idx


def expand_rows(mu_x: np.ndarray, path: np.ndarray) -> np.ndarray:
    """attn^T @ mu_x as the reference computes it (matcha_tts.py:314-315): [B,C,Ty], float64 sums."""
    return np.einsum("bxy,bcx->bcy", np.asarray(path, np.float64), np.asarray(mu_x, np.float64))
