"""ctypes binding of libmtts_hip.so (C ABI: include/mtts.h, include/mtts_decoder.h).

The product path has no fallback: if the library is missing or was built without a symbol, every
op raises.  ``lib()`` loads lazily so that importing the package on a machine without a GPU (CI,
CPU tests) stays cheap; loading itself never touches the GPU.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

_PKG_ROOT = Path(__file__).resolve().parent.parent
LIB_PATH = Path(os.environ.get("MTTS_LIB", _PKG_ROOT / "lib" / "libmtts_hip.so"))

MTTS_OK = 0
MTTS_MAS_VALUE_PREMASKED = 0x1
MTTS_MAS_NO_DENSE_PATH = 0x2
MTTS_MAS_MAX_TX = 8192  # include/mtts.h (maximum_path, prior_maximum_path)
MTTS_MAS_MAX_TX_ROW_MAJOR = 4096  # include/mtts.h (compute_batch_alignments)

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F = ctypes.c_float
_SZ = ctypes.c_size_t

# name -> (restype, argtypes).  Kept in the same order as the header declarations.
_SIGNATURES: dict[str, tuple] = {
    "mtts_abi_version": (ctypes.c_int, []),
    "mtts_last_error": (ctypes.c_char_p, []),
    "mtts_maximum_path_workspace_size": (_SZ, [_I32, _I32, _I32]),
    "mtts_maximum_path_f32": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _I32, _I32, _P, _P, _P, _SZ, _P]),
    "mtts_prior_maximum_path_workspace_size": (_SZ, [_I32, _I32, _I32]),
    "mtts_prior_maximum_path": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _I32, _P, _P, _P, _P, _P, _P, _P,
                                               _SZ, _P]),
    "mtts_expand_rows_fwd": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _I32, _P, _P]),
    "mtts_expand_rows_bwd": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _I32, _I32, _P, _P]),
    "mtts_compute_batch_alignments": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _F, _P, _SZ, _P]),
    "mtts_losses_workspace_size": (_SZ, [_I32, _I32]),
    "mtts_losses_fwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _F, _P, _P, _SZ, _P]),
    "mtts_losses_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _I32, _I32, _F, _P, _P, _P]),
    "mtts_cfm_pack_fwd": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _F, _P, _P]),
    "mtts_cfm_pack_bwd": (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _P]),
    "mtts_time_embedding": (ctypes.c_int, [_P, _I32, _I32, _F, _P, _P]),
    "mtts_mel_log_fwd": (ctypes.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _I32, _F, _P, _P]),
}

_lib = None


class NativeError(RuntimeError):
    pass


def register(name: str, restype, argtypes) -> None:
    """Lets op modules declare the signatures of the entry points they bind."""
    _SIGNATURES[name] = (restype, argtypes)
    if _lib is not None:
        _bind(_lib, name)


def _bind(handle, name):
    fn = getattr(handle, name)
    fn.restype, fn.argtypes = _SIGNATURES[name]


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise NativeError(
                f"{LIB_PATH} not found: build it with `python {_PKG_ROOT / 'build_native.py'}` "
                "(hipcc --offload-arch=gfx950). There is no non-HIP fallback.")
        handle = ctypes.CDLL(str(LIB_PATH))
        for name in _SIGNATURES:
            _bind(handle, name)
        _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != MTTS_OK:
        msg = lib().mtts_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed with status {rc}: {msg}")


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(*tensors: torch.Tensor) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise NativeError("the MI355X hot path takes device (cuda/hip) tensors only; "
                              f"got a tensor on {t.device}")
