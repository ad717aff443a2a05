"""The C-ABI library loads and exports every symbol include/*.h declares; argument validation and
size queries work without a GPU (no compute is launched here)."""
from __future__ import annotations

import ctypes
import re
from pathlib import Path

import pytest

from matcha import _native as N

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols() -> list[str]:
    names = []
    for h in sorted((ROOT / "include").glob("*.h")):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names += re.findall(r"\b(mtts_[a-z0-9_]+)\s*\(", text)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    lib = N.lib()
    syms = declared_symbols()
    assert "mtts_maximum_path_f32" in syms and len(syms) >= 5
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, f"declared in include/*.h but not exported: {missing}"


def test_every_declared_symbol_has_a_python_signature():
    import matcha.models.components._ops  # noqa: F401  (registers the decoder entry points)
    import matcha.training  # noqa: F401  (registers the clip + AdamW entry points)
    import matcha.dp  # noqa: F401  (registers the RCCL data-parallel entry points)
    import matcha.models.components.text_encoder  # noqa: F401  (registers the embedding entry points)

    missing = [s for s in declared_symbols() if s not in N._SIGNATURES]
    assert not missing, missing


def test_abi_version_and_error_slot():
    lib = N.lib()
    assert lib.mtts_abi_version() == 1
    rc = lib.mtts_maximum_path_f32(None, None, None, 2, 0, 5, 0, None, None, None, 0, None)
    assert rc == -1  # MTTS_ERR_INVALID_ARG, before any HIP call
    assert b"bad shape" in lib.mtts_last_error()
    rc = lib.mtts_maximum_path_f32(None, None, None, 2, 4097, 5, 0, None, None, None, 0, None)
    assert rc == -2  # MTTS_ERR_SHAPE: Tx > MTTS_MAS_MAX_TX (4096)
    rc = lib.mtts_maximum_path_f32(None, None, None, 2, 5, 5, 0x80, None, None, None, 0, None)
    assert rc == -1  # unknown flag
    rc = lib.mtts_maximum_path_f32(ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16),
                                   2, 5, 5, 0, None, None, None, 0, None)
    assert rc == -3  # workspace too small
    assert lib.mtts_maximum_path_f32(None, None, None, 0, 5, 5, 0, None, None, None, 0, None) == 0


@pytest.mark.parametrize("B,Tx,Ty", [(1, 1, 1), (32, 120, 600), (8, 512, 4096), (3, 65, 33)])
def test_workspace_size(B, Tx, Ty):
    n = N.lib().mtts_maximum_path_workspace_size(B, Tx, Ty)
    assert n >= B * 2 * 4 + B * Tx * 4
    if Tx == 512:  # backpointer words spill from LDS to the workspace
        assert n >= B * 512 * (Ty // 32) * 4


def test_product_path_refuses_cpu_tensors():
    import torch
    from matcha.utils.monotonic_align import maximum_path

    with pytest.raises(N.NativeError):
        maximum_path(torch.zeros(1, 2, 3), torch.ones(1, 2, 3))
