"""ctypes binding of the CPU oracle (oracle/libmas_oracle.so) -- test infrastructure only.

Builds the oracle with `make -C oracle` on first use if the .so is missing (gcc is present on both
the dev container and the GPU box).
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
SO = ROOT / "oracle" / "libmas_oracle.so"
_P = ctypes.c_void_p
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not SO.exists():
            subprocess.run(["make", "-C", str(ROOT / "oracle")], check=True, capture_output=True)
        _lib = ctypes.CDLL(str(SO))
        _lib.mtts_oracle_mas_batch.argtypes = [_P, _P, _P, _P] + [ctypes.c_int] * 3 + [ctypes.c_float, ctypes.c_int]
        _lib.mtts_oracle_maximum_path.argtypes = [_P] * 6 + [ctypes.c_int] * 4
    return _lib


def _p(a):
    return a.ctypes.data_as(_P)


def mas_batch(values: np.ndarray, t_x: np.ndarray, t_y: np.ndarray, neg: float = -1e9, threads: int = 0):
    """compute_batch_alignments restated (core.pyx:101-128): returns (paths int32, mutated values)."""
    values = np.ascontiguousarray(values, np.float32).copy()
    B, Tx, Ty = values.shape
    paths = np.zeros((B, Tx, Ty), np.int32)
    t_x = np.ascontiguousarray(t_x, np.int32)
    t_y = np.ascontiguousarray(t_y, np.int32)
    rc = lib().mtts_oracle_mas_batch(_p(paths), _p(values), _p(t_x), _p(t_y), B, Tx, Ty, neg, threads)
    assert rc == 0
    return paths, values


def maximum_path(value: np.ndarray, mask: np.ndarray, threads: int = 0):
    """maximum_path restated (__init__.py:40-55): returns (path float32, lengths int32 [B,2])."""
    value = np.ascontiguousarray(value, np.float32)
    mask = np.ascontiguousarray(mask, np.float32)
    B, Tx, Ty = value.shape
    path = np.empty((B, Tx, Ty), np.float32)
    scratch = np.empty((B, Tx, Ty), np.float32)
    iscratch = np.empty((B, Tx, Ty), np.int32)
    t = np.empty((B, 2), np.int32)
    rc = lib().mtts_oracle_maximum_path(_p(value), _p(mask), _p(path), _p(scratch), _p(iscratch), _p(t),
                                        B, Tx, Ty, threads)
    assert rc == 0
    return path, t


def row_start_to_path(rs: np.ndarray, t_x: np.ndarray, t_y: np.ndarray, Ty: int) -> np.ndarray:
    """Expands int32 row starts [B,Tx] into the dense {0,1} path [B,Tx,Ty] (int8)."""
    B, Tx = rs.shape
    out = np.zeros((B, Tx, Ty), np.int8)
    for b in range(B):
        for x in range(Tx):
            s = rs[b, x]
            if s < 0:
                continue
            e = t_y[b] - 1 if x == t_x[b] - 1 else rs[b, x + 1] - 1
            out[b, x, s : e + 1] = 1
    return out


def lengths_mask(B, Tx, Ty, t_x, t_y) -> np.ndarray:
    m = np.zeros((B, Tx, Ty), np.float32)
    for b in range(B):
        m[b, : t_x[b], : t_y[b]] = 1.0
    return m
