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
    import matcha.watchdog  # noqa: F401  (registers the device progress markers)
    import matcha.models.components.text_encoder  # noqa: F401  (registers the embedding entry points)

    missing = [s for s in declared_symbols() if s not in N._SIGNATURES]
    assert not missing, missing


def test_abi_version_and_error_slot():
    lib = N.lib()
    assert lib.mtts_abi_version() == 1
    rc = lib.mtts_maximum_path_f32(None, None, None, 2, 0, 5, 0, None, None, None, 0, None)
    assert rc == -1  # MTTS_ERR_INVALID_ARG, before any HIP call
    assert b"bad shape" in lib.mtts_last_error()
    rc = lib.mtts_maximum_path_f32(None, None, None, 2, 8193, 5, 0, None, None, None, 0, None)
    assert rc == -2  # MTTS_ERR_SHAPE: Tx > MTTS_MAS_MAX_TX (8192)
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


def test_gemm_workspace_query_plans_the_schedule_that_runs():
    """mtts_conv_gemm_workspace_size resolves the operand-driven schedule rewrites the launch applies:
    the bf16x6 text-encoder prenet (3840 x 192, k = 5 over 192 channels, three weight planes) runs the LDS-DMA
    64 x 64 schedule with split K, so its size query must ask for the split slabs (it returned 0 when it planned
    the raw heuristic's register config, and the launch then ran unsplit)."""
    from matcha.models.components import _ops as O

    a = O.ConvGemmArgs()
    a.A, a.W, a.C = 4096, 8192, 12288  # 16-byte aligned placeholders: size queries dereference nothing
    a.lda, a.Ti, a.To, a.nb, a.in_stride, a.ntaps, a.cin = 192, 120, 120, 32, 1, 5, 192
    for j in range(5):
        a.off[j] = j - 2
    a.N, a.K, a.Kp = 192, 960, 960
    a.ldc, a.To_full, a.out_stride = 192, 120, 1
    a.flags = O.GEMM_F_SPLIT3
    ws = N.lib().mtts_conv_gemm_workspace_size(ctypes.byref(a), O.PREC_BF16, -1, 0)
    assert ws == 2 * 3840 * 192 * 4, ws  # two fp32 partial slabs of M x N
    a.flags = 0  # one plane: the register schedule, no split
    assert N.lib().mtts_conv_gemm_workspace_size(ctypes.byref(a), O.PREC_BF16, -1, 0) == 0
