"""Token-major ([B, T, C], C contiguous) device operators of the CFM decoder.

The reference runs the decoder channel-major ([B, C, T]) and rearranges to [B, T, C] around every
transformer block (decoder.py:298-306, 324-332, 345-353).  Here activations stay token-major for the
whole U-Net: a k-tap Conv1d is an implicit GEMM over K = k*C_in with rows = tokens, the transformer
GEMMs need no transposes, and the reference's rearranges disappear.

Every operator is a torch.autograd.Function whose forward AND backward run in libmtts_hip.so
(include/mtts_decoder.h); there is no fallback -- without the library (or on CPU tensors) they raise.
  conv_tm / conv_transpose_tm / linear_tm / ff_tm  -> mtts_conv_gemm + mtts_conv_wgrad
      (stride-2 conv dgrad and the ConvTranspose1d forward run as two "phase" GEMMs; the transposed
       conv's dgrad is a stride-2 conv)
  group_norm_mish_tm                               -> mtts_gn_mish_fwd / _bwd
  layer_norm_tm                                    -> mtts_layernorm_fwd / _bwd
  attention_tm                                     -> mtts_attention_fwd / _bwd (flash attention)
GEMM precision follows the caller: inside a bf16 torch.autocast region the GEMMs use bf16 MFMA with
fp32 accumulation, otherwise exact-fp32 MFMA (the parity mode).  Activations stay fp32 in HBM.
Dropout (train mode) is a counter-based mask generated in the GEMM epilogues and regenerated in the
backward, so no mask tensor is stored.
"""
from __future__ import annotations

import contextlib
import contextvars
import ctypes
import functools
import os
import math

import torch
import torch.nn.functional as F

from matcha import _native as N

PREC_FP32, PREC_BF16 = 0, 1
ACT_NONE, ACT_GELU, ACT_DGELU, ACT_RELU, ACT_DRELU = 0, 1, 2, 3, 4

KERNELS: dict[str, str] = {
    "conv_tm": "mtts_conv_gemm/mtts_conv_wgrad",
    "conv_transpose_tm": "mtts_conv_gemm/mtts_conv_wgrad",
    "linear_tm": "mtts_conv_gemm/mtts_conv_wgrad",
    "ff_tm": "mtts_conv_gemm/mtts_conv_wgrad",
    "group_norm_mish_tm": "mtts_gn_mish_fwd/mtts_gn_mish_bwd",
    "layer_norm_tm": "mtts_layernorm_fwd/mtts_layernorm_bwd",
    "conv_ffn_tm": "mtts_conv_gemm/mtts_conv_wgrad/mtts_act_dropout_bwd",
    "rope_tm": "mtts_rope_qk",
    "attention_tm": "mtts_attention_fwd/mtts_attention_bwd",
}


GEMM_F_BINARY_SCALE = 0x1  # include/mtts_decoder.h MTTS_GEMM_F_BINARY_SCALE
GEMM_F_A_BF16 = 0x2  # MTTS_GEMM_F_A_BF16: A operand stored bf16 (bf16-mixed activations)
GEMM_F_C_BF16 = 0x4  # MTTS_GEMM_F_C_BF16: output stored bf16
GEMM_F_FAST_ACT = 0x8  # MTTS_GEMM_F_FAST_ACT: 1.5e-7-accurate erf in GELU epilogues (bf16-mixed only)
GEMM_F_PRE_BF16 = 0x10  # MTTS_GEMM_F_PRE_BF16: C_pre written / aux read as bf16
WGRAD_F_DY_BF16 = 0x20  # MTTS_WGRAD_F_DY_BF16: the weight gradient's dY holds bf16
GEMM_F_W_SPLIT = 0x40  # MTTS_GEMM_F_W_SPLIT: W holds a hi and a lo bf16 plane (two MFMAs per product)
_FAST_ACT = os.environ.get("MTTS_EXACT_GELU") != "1"
# Weight planes of the bf16-mixed forward GEMMs.  Split (two bf16 planes, hi + rounding residual): the
# rounding of the fp32 weights is a static model perturbation and is the bf16 loss error
# (tools/r3/precision_budget.py: prior 2.9e-4 / diff 2.1e-4 from weight rounding alone, activations
# 3.8e-5 / 2.1e-5 at B=32) -- with split planes bf16-mixed meets the 1e-4 loss bar at the bench batch, at
# ~+50 % forward-GEMM time (bench.py reports both lines).  Default one plane (the throughput mode);
# MTTS_W_SPLIT=1 or set_weight_split(True) selects the split planes.
_W_SPLIT = os.environ.get("MTTS_W_SPLIT", "0") == "1"


GEMM_F_A_SPLIT = 0x80  # MTTS_GEMM_F_A_SPLIT: with W_SPLIT, fp32 A split into hi + lo planes (bf16x3)
# precise_forward(): inside a bf16-mixed region, the forward GEMMs take split weight planes AND split A
# operands (A_hi W_hi + A_hi W_lo + A_lo W_hi: ~16 significant bits per operand, fp32 accumulate) and the
# attention forward runs exact fp32 MFMA; the backward of the same ops stays bf16 one-plane.  The
# text encoder runs this way in the parity policy (MatchaTTS.encoder_precision = "bf16x3"): its
# activations' bf16 rounding decides the alignment's near-ties (tools/r3/precision_budget.py).
_PRECISE: contextvars.ContextVar = contextvars.ContextVar("mtts_precise_fwd", default=False)


@contextlib.contextmanager
def precise_forward(on: bool | str = True):
    """on: True / "bf16x3" (split bf16 operands, three MFMAs per product), "bf16x6" (three exact planes per
    operand, six MFMAs per product: fp32-faithful, MTTS_GEMM_F_SPLIT3) or "fp32" (the forward GEMMs on the
    exact-fp32 MFMA with fp32 packed weights -- the 32-true arithmetic, so the forward's outputs are those of
    32-true; round 4: bf16x3 left one alignment near-tie of the B=4 reference fixture flipped); False: off.
    The backward of the same ops stays bf16 one-plane either way."""
    tok = _PRECISE.set(("bf16x3" if on is True else on) if on else False)
    try:
        yield
    finally:
        _PRECISE.reset(tok)


def _fwd_fp32() -> bool:
    """precise_forward("fp32") is active: bf16-region forward GEMMs run as exact fp32."""
    return _PRECISE.get() == "fp32"


def set_weight_split(on: bool) -> bool:
    """Selects one (False) or two (True) bf16 weight planes for the bf16-mixed forward GEMMs from the next
    forward on; returns the previous setting.  (Captured graphs keep the packing they were captured with.)"""
    global _W_SPLIT
    old, _W_SPLIT = _W_SPLIT, bool(on)
    return old


_WSPLIT_CV: contextvars.ContextVar = contextvars.ContextVar("mtts_w_split", default=None)
# the text encoder's precision inside bf16-mixed when the model does not set its own
# (MatchaTTS.encoder_precision): "bf16", "bf16x3" / "bf16x6" / "fp32fwd" (precise_forward) or "fp32"
_ENC_PREC: contextvars.ContextVar = contextvars.ContextVar("mtts_encoder_precision", default="bf16")


def weight_split_enabled() -> bool:
    v = _WSPLIT_CV.get()
    return _W_SPLIT if v is None else v


# The decoder FeedForward's GELU up-projection keeps ONE bf16 weight plane under the parity policy: its share of the
# diffusion loss's weight-rounding error is ~3.5 % (tools/r3/weight_sensitivity.py), and its split planes cost the
# most of any GEMM (the GELU epilogue pins it to the register schedule).  Measured (profiles/r04/ff1_one_plane/):
# step 7.99 / 8.01 -> 7.85 / 7.86 ms; parity errors (prior, diff) B=4 vs the reference fixture 0 / 1.2e-5, B=32
# 0 / 3.4e-7, 512 x 4096 1.9e-7 / 3.3e-5, alignment exact in all three.  MTTS_PARITY_FF1_SPLIT=1: split it too.
_FF1_SPLIT = os.environ.get("MTTS_PARITY_FF1_SPLIT", "0") != "0"
# MTTS_PARITY_FF2_SPLIT=0: the FF down-projection in one plane too (~3 % share; A/B only)
_FF2_SPLIT = os.environ.get("MTTS_PARITY_FF2_SPLIT", "1") != "0"

# the parity policy's text-encoder forward: "fp32fwd" (exact-fp32 MFMA: 32-true's arithmetic) or "bf16x6"
# (three exact bf16 planes per operand, six MFMAs).  bf16x6 measured 8.16 vs 8.05 ms per step and 1-3x the
# fp32 kernel's error, enough to move 2 of 437 durations at B=4 (profiles/r04/x6): fp32fwd stays the
# default; MTTS_PARITY_ENCODER selects
_PARITY_ENC = os.environ.get("MTTS_PARITY_ENCODER", "fp32fwd")


def encoder_precision_for_parity() -> str:
    return _PARITY_ENC


@contextlib.contextmanager
def parity_policy(on: bool = True):
    """bf16-parity inside a bf16 autocast region (the Trainer's "bf16-parity" precision): split weight
    planes for every forward GEMM but the decoder FeedForward's GELU up-projection (_FF1_SPLIT) and the text
    encoder's forward on the exact-fp32 MFMA
    (precise_forward("fp32"); its backward stays bf16)."""
    t1 = _WSPLIT_CV.set(True if on else None)
    t2 = _ENC_PREC.set(_PARITY_ENC if on else "bf16")
    try:
        yield
    finally:
        _ENC_PREC.reset(t2)
        _WSPLIT_CV.reset(t1)


def encoder_precision_default() -> str:
    return _ENC_PREC.get()
PACK_BF16_SPLIT = 2  # pack-cache kind: the bf16 hi + lo planes of a forward operand
PACK_BF16_SPLIT3 = 3  # pack-cache kind: hi + mid + lo bf16 planes (== w exactly) of a bf16x6 forward operand
GEMM_F_SPLIT3 = 0x100  # MTTS_GEMM_F_SPLIT3: three weight planes, fp32 A split in the kernel (bf16x6)
PACK_THREE_PLANES = 1 << 62  # MTTS_PACK_THREE_PLANES (mtts_pack_job.lo_off flag)

GEMM_GLDS = 32  # MTTS_GEMM_GLDS: first LDS-DMA schedule id


class ConvGemmArgs(ctypes.Structure):
    _fields_ = [("A", ctypes.c_void_p), ("a_scale", ctypes.c_void_p), ("lda", ctypes.c_int32),
                ("Ti", ctypes.c_int32), ("To", ctypes.c_int32), ("nb", ctypes.c_int32),
                ("in_stride", ctypes.c_int32), ("ntaps", ctypes.c_int32), ("off", ctypes.c_int32 * 8),
                ("cin", ctypes.c_int32), ("W", ctypes.c_void_p), ("N", ctypes.c_int32), ("K", ctypes.c_int32),
                ("Kp", ctypes.c_int32), ("bias", ctypes.c_void_p), ("act", ctypes.c_int32),
                ("residual", ctypes.c_void_p), ("ldr", ctypes.c_int32), ("c_scale", ctypes.c_void_p),
                ("C", ctypes.c_void_p), ("ldc", ctypes.c_int32), ("To_full", ctypes.c_int32),
                ("out_stride", ctypes.c_int32), ("out_off", ctypes.c_int32), ("C_pre", ctypes.c_void_p),
                ("aux", ctypes.c_void_p), ("ldaux", ctypes.c_int32), ("dropout_p", ctypes.c_float),
                ("seed", ctypes.c_void_p), ("flags", ctypes.c_int32)]


class ConvWgradArgs(ctypes.Structure):
    _fields_ = [("dY", ctypes.c_void_p), ("ldy", ctypes.c_int32), ("To_full", ctypes.c_int32),
                ("out_stride", ctypes.c_int32), ("out_off", ctypes.c_int32), ("A", ctypes.c_void_p),
                ("a_scale", ctypes.c_void_p), ("lda", ctypes.c_int32), ("Ti", ctypes.c_int32),
                ("To", ctypes.c_int32), ("nb", ctypes.c_int32), ("in_stride", ctypes.c_int32),
                ("ntaps", ctypes.c_int32), ("off", ctypes.c_int32 * 8), ("cin", ctypes.c_int32),
                ("N", ctypes.c_int32), ("K", ctypes.c_int32), ("flags", ctypes.c_int32)]


class AttnArgs(ctypes.Structure):
    _fields_ = [("q", ctypes.c_void_p), ("k", ctypes.c_void_p), ("v", ctypes.c_void_p), ("ldq", ctypes.c_int32),
                ("key_bias", ctypes.c_void_p), ("o", ctypes.c_void_p), ("ldo", ctypes.c_int32),
                ("lse", ctypes.c_void_p), ("B", ctypes.c_int32), ("T", ctypes.c_int32), ("H", ctypes.c_int32),
                ("D", ctypes.c_int32), ("scale", ctypes.c_float), ("dropout_p", ctypes.c_float),
                ("seed", ctypes.c_void_p), ("flags", ctypes.c_int32)]
ATTN_F_IO_BF16 = 0x1  # include/mtts_decoder.h MTTS_ATTN_F_IO_BF16


class AttnGrads(ctypes.Structure):
    _fields_ = [("dout", ctypes.c_void_p), ("lddo", ctypes.c_int32), ("dq", ctypes.c_void_p),
                ("dk", ctypes.c_void_p), ("dv", ctypes.c_void_p), ("ldd", ctypes.c_int32)]


class PackJob(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("rows", ctypes.c_int32), ("C", ctypes.c_int32),
                ("ntaps", ctypes.c_int32), ("Kp", ctypes.c_int32), ("ld", ctypes.c_int32), ("sr", ctypes.c_int64),
                ("sc", ctypes.c_int64), ("sj", ctypes.c_int64), ("j0", ctypes.c_int32), ("js", ctypes.c_int32),
                ("lo_off", ctypes.c_int64)]


_P, _I, _F, _SZ, _U = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float, ctypes.c_size_t, ctypes.c_uint32
_I64 = ctypes.c_int64
N.register("mtts_conv_gemm", ctypes.c_int, [ctypes.POINTER(ConvGemmArgs), _I, _P])
N.register("mtts_conv_gemm_tile", ctypes.c_int, [ctypes.POINTER(ConvGemmArgs), _I, _I, _P])
N.register("mtts_conv_gemm_workspace_size", _SZ, [ctypes.POINTER(ConvGemmArgs), _I, _I, _I])
N.register("mtts_conv_gemm_ws", ctypes.c_int, [ctypes.POINTER(ConvGemmArgs), _I, _I, _I, _P, _SZ, _P])
N.register("mtts_conv_wgrad_workspace_size", _SZ, [ctypes.POINTER(ConvWgradArgs)])
N.register("mtts_conv_wgrad", ctypes.c_int,
           [ctypes.POINTER(ConvWgradArgs), _I, _P, _I64, _I64, _I64, _P, _I, _P, _SZ, _P])
N.register("mtts_conv_wgrad_tile", ctypes.c_int,
           [ctypes.POINTER(ConvWgradArgs), _I, _I, _I, _I, _P, _I64, _I64, _I64, _P, _I, _P, _SZ, _P])
N.register("mtts_gn_mish_fwd", ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _P])
N.register("mtts_gn_mish_bwd_workspace_size", _SZ, [_I, _I])
N.register("mtts_gn_mish_bwd", ctypes.c_int,
           [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _SZ, _P])
N.register("mtts_gn_mish_fwd_ex", ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _F, _I, _P])
N.register("mtts_gn_mish_bwd_ex", ctypes.c_int,
           [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P])
NORM_F_X_BF16, NORM_F_DY_BF16 = 0x200, 0x400  # include/mtts_decoder.h
N.register("mtts_layernorm_fwd", ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I, _I, _F, _I, _F, _P, _P])
N.register("mtts_layernorm_bwd_workspace_size", _SZ, [_I, _I])
N.register("mtts_layernorm_bwd", ctypes.c_int,
           [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _P, _P, _SZ, _P])
N.register("mtts_dropout_apply", ctypes.c_int, [_P, _P, _I, _I, _I, _F, _P, _P])
N.register("mtts_act_dropout_bwd", ctypes.c_int, [_P, _P, _P, _I, _I, _I, _I, _F, _P, _P])
N.register("mtts_act_dropout_bwd_scaled", ctypes.c_int, [_P, _P, _P, _P, _I, _I, _I, _I, _F, _P, _P])
N.register("mtts_rope_qk", ctypes.c_int, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _I, _P])
N.register("mtts_pack_weights", ctypes.c_int, [ctypes.POINTER(PackJob), _I, _I, _P])
N.register("mtts_attention_fwd", ctypes.c_int, [ctypes.POINTER(AttnArgs), _I, _P])
N.register("mtts_attention_bwd_workspace_size", _SZ, [_I, _I, _I])
N.register("mtts_attention_bwd", ctypes.c_int, [ctypes.POINTER(AttnArgs), ctypes.POINTER(AttnGrads), _I, _P, _SZ, _P])
N.register("mtts_reduce_partials", ctypes.c_int, [_P, _I, _P])
N.register("mtts_defer_reductions", None, [_I])
N.register("mtts_pending_reductions", _I, [])
N.register("mtts_flush_reductions", ctypes.c_int, [_P])
N.register("mtts_discard_reductions", None, [])
N.register("mtts_wgrad_plan_mode", None, [_I])
N.register("mtts_wgrad_flush_cap", None, [_I])
N.register("mtts_colsum_workspace_size", _SZ, [_I64, _I])
N.register("mtts_colsum", ctypes.c_int, [_P, _I64, _I, _I, _P, _I, _P, _SZ, _P])


# ------------------------------------------------------------------------------------------ helpers
def gemm_precision() -> int:
    """bf16 MFMA inside a bf16 autocast region, exact-fp32 MFMA otherwise."""
    if torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16:
        return PREC_BF16
    return PREC_FP32


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _f32c(t: torch.Tensor | None) -> torch.Tensor | None:
    if t is None:
        return None
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def _actc(t: torch.Tensor | None, prec: int) -> torch.Tensor | None:
    """An activation as the kernels take it: bf16 stays bf16 in bf16-mixed mode (a GEMM A operand /
    GroupNorm input stored as autocast would hold it), anything else becomes contiguous fp32."""
    if t is not None and t.dtype == torch.bfloat16 and prec == PREC_BF16:
        return t.contiguous()
    return _f32c(t)


def _bf16_operand_ok(c: int) -> bool:
    """A bf16 A operand needs the LDS-DMA schedules: >= 64 channels, rows of whole 16-byte chunks."""
    return c >= 64 and c % 8 == 0


_SEED_SCOPE: contextvars.ContextVar = contextvars.ContextVar("mtts_seed_scope", default=None)


def _new_seed(device) -> torch.Tensor:
    """Two random words drawn ON THE DEVICE from torch's generator: no host sync, and a captured
    HIP graph draws fresh dropout masks on every replay (torch's graph-safe philox offsets).  Inside
    a weight_pack_scope the words are slices of ONE pool drawn when the scope opens (sized by the
    owner's previous forward): one generator launch per module forward instead of one per dropout."""
    st = _SEED_SCOPE.get()
    if st is not None:
        st["used"] += 1
        pool = st["pool"]
        if pool is not None and pool.device == torch.device(device) and st["i"] + 2 <= pool.numel():
            i = st["i"]
            st["i"] = i + 2
            return pool[i:i + 2]
    return torch.randint(0, 2 ** 31 - 1, (2,), device=device, dtype=torch.int32)


def pack_weight(w2d: torch.Tensor, prec: int) -> tuple[torch.Tensor, int]:
    """[N, K] -> contiguous [N, Kp] (Kp = K rounded up to 8) in the GEMM's operand precision."""
    N_, K = w2d.shape
    Kp = (K + 7) // 8 * 8
    w = w2d.detach().to(torch.bfloat16 if prec == PREC_BF16 else torch.float32)
    if Kp != K:
        w = F.pad(w, (0, Kp - K))
    return w.contiguous(), Kp


# ------------------------------------------------------------------------------------------ weight packing
# A GEMM operand layout of one or more fp32 weights: [rows][Kp] in the operand precision, built by
# mtts_pack_weights jobs (include/mtts_decoder.h).  job = (src, row0, rows, col0, Kp_job, C, ntaps,
# sr, sc, sj, j0, js): dst[row0 + r][col0 + j*C + c] = src[r*sr + c*sc + (j0 + j*js)*sj].
class PackSpec:
    __slots__ = ("key", "rows", "Kp", "jobs", "dgrad", "one_plane")

    def __init__(self, key, rows, Kp, jobs, dgrad, one_plane=False):
        self.key, self.rows, self.Kp, self.jobs, self.dgrad = key, rows, Kp, jobs, dgrad
        self.one_plane = one_plane  # a forward operand kept in one bf16 plane even where the policy splits


def _r8(n):
    return (n + 7) // 8 * 8


def spec_linear(ws, dgrad=False, one_plane=False):
    """Linear weights [N_i, K] stacked along N -> [sum N_i, Kp] (forward); dgrad: the transpose
    [K, sum N_i] (column blocks; each N_i % 8 == 0 when stacking).  one_plane: never the split planes."""
    ws = tuple(ws)
    K = ws[0].shape[1]  # nn.Conv1d 1x1 weights [N, K, 1] have the Linear layout
    if not dgrad:
        jobs, r0 = [], 0
        for w in ws:
            jobs.append((w, r0, w.shape[0], 0, _r8(K), K, 1, K, 1, 0, 0, 1))
            r0 += w.shape[0]
        return PackSpec(("lin",) + tuple(id(w) for w in ws), r0, _r8(K), jobs, False, one_plane)
    ntot = sum(w.shape[0] for w in ws)
    jobs, c0 = [], 0
    for i, w in enumerate(ws):
        last = i == len(ws) - 1
        jobs.append((w, 0, K, c0, (_r8(ntot) - c0) if last else w.shape[0], w.shape[0], 1, 1, K, 0, 0, 1))
        c0 += w.shape[0]
    return PackSpec(("lin_t",) + tuple(id(w) for w in ws), K, _r8(ntot), jobs, True)


def spec_conv_fwd(w):
    """Conv1d weight [Cout, Cin, k] -> [Cout][j*Cin + c]."""
    Cout, Cin, k = w.shape
    return PackSpec(("conv", id(w)), Cout, _r8(k * Cin), [(w, 0, Cout, 0, _r8(k * Cin), Cin, k, Cin * k, k, 1, 0, 1)],
                    False)


def spec_conv_dgrad(w, j0=0, js=1):
    """Conv1d dgrad operand: [Cin][jj*Cout + n] = w[n, c, j0 + jj*js] (all taps, or one stride phase)."""
    Cout, Cin, k = w.shape
    nt = len(range(j0, k, js))
    return PackSpec(("conv_d", id(w), j0, js), Cin, _r8(nt * Cout),
                    [(w, 0, Cin, 0, _r8(nt * Cout), Cout, nt, k, Cin * k, 1, j0, js)], True)


def spec_convT_fwd(w, j0, js):
    """ConvTranspose1d weight [Cin, Cout, k], output phase taps j0::js -> [Cout][jj*Cin + c]."""
    Cin, Cout, k = w.shape
    nt = len(range(j0, k, js))
    return PackSpec(("convT", id(w), j0, js), Cout, _r8(nt * Cin),
                    [(w, 0, Cout, 0, _r8(nt * Cin), Cin, nt, k, Cout * k, 1, j0, js)], False)


def spec_convT_dgrad(w):
    """ConvTranspose1d dgrad operand (a stride-2 conv over dy): [Cin][j*Cout + n] = w[c, n, j]."""
    Cin, Cout, k = w.shape
    return PackSpec(("convT_d", id(w)), Cin, _r8(k * Cout), [(w, 0, Cin, 0, _r8(k * Cout), Cout, k, Cout * k, k, 1, 0, 1)],
                    True)


def _run_pack(specs, prec, stream=None):
    """prec: PREC_FP32, PREC_BF16, PACK_BF16_SPLIT ([2 * rows, Kp]: the hi plane, then the lo plane) or
    PACK_BF16_SPLIT3 ([3 * rows, Kp]: hi, mid, lo).
    stream: launch there instead of the current stream (outputs are allocated on the current one)."""
    dev = specs[0].jobs[0][0].device
    split3 = prec == PACK_BF16_SPLIT3
    split = prec == PACK_BF16_SPLIT or split3
    dt = torch.bfloat16 if prec in (PREC_BF16, PACK_BF16_SPLIT, PACK_BF16_SPLIT3) else torch.float32
    outs = [torch.empty((3 if split3 else 2 if split else 1) * sp.rows, sp.Kp, device=dev, dtype=dt) for sp in specs]
    njobs = sum(len(sp.jobs) for sp in specs)
    arr = (PackJob * njobs)()
    i = 0
    keep = []
    for sp, out in zip(specs, outs):
        es = out.element_size()
        for (w, r0, rows, c0, kpj, C, nt, sr, sc, sj, j0, js) in sp.jobs:
            src = _f32c(w)
            keep.append(src)
            j = arr[i]
            j.src, j.dst = src.data_ptr(), out.data_ptr() + (r0 * sp.Kp + c0) * es
            j.rows, j.C, j.ntaps, j.Kp, j.ld = rows, C, nt, kpj, sp.Kp
            j.sr, j.sc, j.sj, j.j0, j.js = sr, sc, sj, j0, js
            j.lo_off = (sp.rows * sp.Kp if split else 0) | (PACK_THREE_PLANES if split3 else 0)
            i += 1
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    N.check(N.lib().mtts_pack_weights(arr, njobs, PREC_BF16 if split else prec, st.cuda_stream), "mtts_pack_weights")
    if split3:
        for o in outs:
            o._mtts_w_split3 = True  # _gemm sets MTTS_GEMM_F_SPLIT3 for it
    elif split:
        for o in outs:
            o._mtts_w_split = True  # _gemm sets MTTS_GEMM_F_W_SPLIT for it
    return outs


def _pack_kind(spec: PackSpec, prec: int) -> int:
    """bf16 forward operands: fp32 under precise_forward("fp32"), the split planes when selected
    (set_weight_split, precise_forward("bf16x3")); everything else as prec."""
    if prec == PREC_BF16 and not spec.dgrad:
        # one_plane is the parity POLICY's choice (parity_policy()); set_weight_split(True) alone splits
        # every forward operand, so its error numbers mean what the mode says
        if spec.one_plane and not _PRECISE.get() and _WSPLIT_CV.get() is not None:
            return prec
        if _fwd_fp32():
            return PREC_FP32
        if _PRECISE.get() == "bf16x6":
            return PACK_BF16_SPLIT3
        if weight_split_enabled() or _PRECISE.get():
            return PACK_BF16_SPLIT
    return prec


_PACK_SCOPE: contextvars.ContextVar = contextvars.ContextVar("mtts_pack_scope", default=None)


@contextlib.contextmanager
def weight_pack_scope(owner: torch.nn.Module):
    """Packs, in a few launches, every operand layout `owner`'s previous forward asked for (the
    backward's transposed layouts too when grad is enabled), and serves the ops inside the scope
    from that cache.  Layouts requested for the first time are packed on demand and remembered."""
    prec = gemm_precision()
    plan = owner.__dict__.setdefault("_mtts_pack_plan", {})
    pre = owner.__dict__.pop("_mtts_pack_pre", None)
    if pre is not None and pre[0] == (prec, torch.is_grad_enabled()):
        cache = pre[1]  # packed ahead on the side stream (prefetch_packs): wait for it
        torch.cuda.current_stream(pre[2].device).wait_stream(pre[2])
    else:
        cache = _pack_plan_now(plan, prec)
    tok = _PACK_SCOPE.set((plan, cache, prec))
    nseed = owner.__dict__.get("_mtts_seed_count", 0)
    dev = next(owner.parameters()).device
    pool = (torch.randint(0, 2 ** 31 - 1, (2 * nseed,), device=dev, dtype=torch.int32)
            if nseed and dev.type == "cuda" else None)
    seeds = {"pool": pool, "i": 0, "used": 0}
    stok = _SEED_SCOPE.set(seeds)
    try:
        yield
    finally:
        _SEED_SCOPE.reset(stok)
        _PACK_SCOPE.reset(tok)
        owner.__dict__["_mtts_seed_count"] = seeds["used"]


def _pack_plan_now(plan, prec, stream=None):
    """Every layout in `plan` for this precision (the backward's transposed ones too when grad is
    enabled), a few launches per kind -> {key: packed}."""
    grad = torch.is_grad_enabled()
    kinds = (prec, PACK_BF16_SPLIT, PACK_BF16_SPLIT3, PREC_FP32) if prec == PREC_BF16 else (prec,)
    cache = {}
    for kind in kinds:
        specs = [sp for key, sp in plan.items()
                 if key[0] == kind and (grad or not sp.dgrad) and _pack_kind(sp, prec) == kind]
        if specs:
            for sp, t in zip(specs, _run_pack(specs, kind, stream)):
                cache[(kind,) + sp.key] = t
    return cache


def prefetch_packs(owner: torch.nn.Module, side) -> None:
    """Packs `owner`'s known layouts NOW on `side` (outputs allocated on the current stream), for its next
    weight_pack_scope -- which waits for `side` and skips its own packing.  The weights must not change
    in between (one forward)."""
    plan = owner.__dict__.get("_mtts_pack_plan")
    if not plan:
        return
    prec = gemm_precision()
    cache = _pack_plan_now(plan, prec, side)
    keep_for_side(*cache.values())  # alive until the side stream is joined, used or not
    owner.__dict__["_mtts_pack_pre"] = ((prec, torch.is_grad_enabled()), cache, side)


def packed(spec: PackSpec, prec: int) -> tuple[torch.Tensor, int]:
    """(operand, Kp) for `spec`, from the active weight_pack_scope when there is one."""
    act = _PACK_SCOPE.get()
    kind = _pack_kind(spec, prec)
    if act is not None and act[2] == prec:
        plan, cache, _ = act
        key = (kind,) + spec.key
        t = cache.get(key)
        if t is None:
            t = _run_pack([spec], kind)[0]
            cache[key] = t
            plan[key] = spec
        return t, spec.Kp
    return _run_pack([spec], kind)[0], spec.Kp


# Per-launch timing for bench.py's roofline leg: when set to a list, every mtts_conv_gemm launch appends
# (start_event, end_event, algorithmic_flops, precision, algorithmic_bytes), events recorded on the
# launch stream.  Algorithmic bytes: the unique input rows once (nb*Ti*cin*4), the packed weights,
# the output, and the residual / aux / pre-activation tensors the epilogue touches.
LAUNCH_LOG: list | None = None
# The same for the weight-gradient GEMMs (mtts_conv_wgrad: partial slabs, and their reduction when it
# runs inside the call) and the attention kernels (mtts_attention_fwd / _bwd): lists of
# (start_event, end_event, algorithmic_flops, precision, algorithmic_bytes, kind).
WGRAD_LOG: list | None = None
ATTN_LOG: list | None = None


def _events(dev):
    st = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    return st, e0, e1


def _ld(t: torch.Tensor) -> int:
    """Row stride (elements) of a GEMM operand: contiguous, or a row-strided view (unit element stride,
    rows ld apart, batches T * ld apart -- e.g. a channel slice of the up path's concat gradient)."""
    if t.dim() < 2 or t.is_contiguous():
        return t.shape[-1]
    if t.dim() > 3 or t.stride(-1) != 1 or (t.dim() == 3 and t.stride(0) != t.shape[1] * t.stride(1)):
        raise ValueError(f"operand layout {tuple(t.shape)} / {t.stride()} is not row-strided")
    return t.stride(-2)


_ROW_STRIDED = os.environ.get("MTTS_ROW_STRIDED", "1") != "0"


def _row_strided_f32(t: torch.Tensor) -> bool:
    if not _ROW_STRIDED:
        return False
    try:
        return t.dtype == torch.float32 and t.dim() == 3 and _ld(t) >= t.shape[-1]
    except ValueError:
        return False


def _gemm(A, Ti, To, nb, in_stride, offs, cin, Wp, Kp, N_, C, To_full, out_stride=1, out_off=0, *, prec,
          a_scale=None, bias=None, act=ACT_NONE, residual=None, c_scale=None, C_pre=None, aux=None,
          dropout_p=0.0, seed=None, tile_cfg=-1, binary_scale=True, splits=0):
    """One mtts_conv_gemm launch.  Every row scale the model passes (a_scale) is a sequence mask
    (matcha.utils.model.sequence_mask: 0/1 by construction, as the reference's x * mask), so
    ``binary_scale`` defaults to True: the bf16 LDS-DMA schedule then reads masked rows as zeros
    instead of multiplying.  Pass False for a general row scale."""
    # host-side shape checks before any launch (the kernel trusts W's rows / the output's extent)
    if Wp.dim() != 2 or Wp.shape[0] < N_ or Wp.shape[1] != Kp or Kp < len(offs) * cin:
        raise ValueError(f"packed weight {tuple(Wp.shape)} does not cover N={N_}, Kp={Kp}, K={len(offs) * cin}")
    if prec == PREC_BF16 and Wp.dtype == torch.float32:
        # precise_forward("fp32"): an fp32-packed forward operand inside a bf16 region runs the exact-fp32
        # MFMA (the 32-true kernels) on fp32 A
        prec = PREC_FP32
        if A.dtype != torch.float32:
            A = A.float()
    w_split = getattr(Wp, "_mtts_w_split", False) and prec == PREC_BF16
    split3 = getattr(Wp, "_mtts_w_split3", False) and prec == PREC_BF16
    if split3:
        if Wp.shape[0] != 3 * N_:
            raise ValueError(f"three weight planes {tuple(Wp.shape)}: the planes must start at rows N={N_}, 2N")
        if A.dtype != torch.float32:
            A = A.float()
    # bf16x3 (precise_forward): the split weights' GEMM also splits its fp32 A operand -- register schedules
    a_split = w_split and _PRECISE.get() and A.dtype == torch.float32
    if a_split:
        tile_cfg, splits = (tile_cfg if 0 <= tile_cfg < GEMM_GLDS else -1), 1
    if w_split and Wp.shape[0] != 2 * N_:
        raise ValueError(f"split weight planes {tuple(Wp.shape)}: the lo plane must start at row N={N_}")
    if C.shape[-1] < N_ or C.numel() < nb * To_full * C.shape[-1] or A.shape[-1] < cin:
        raise ValueError(f"GEMM operands too small: A {tuple(A.shape)}, C {tuple(C.shape)}, N={N_}")
    for t, w_ in ((residual, N_), (aux, N_), (C_pre, N_)):
        if t is not None and (t.shape[-1] < w_ or t.numel() < nb * To_full * t.shape[-1]):
            raise ValueError(f"epilogue operand {tuple(t.shape)} too small for N={N_}")
    # the residual may be a row-strided view (rows ldr apart, e.g. a channel slice of a concat gradient)
    ldr = 0
    if residual is not None:
        ldr = residual.stride(-2) if residual.dim() >= 2 else residual.shape[-1]
        if residual.stride(-1) != 1 or ldr < N_ or (residual.dim() == 3 and residual.stride(0) != residual.shape[1] * ldr):
            raise ValueError(f"residual layout {tuple(residual.shape)} / {residual.stride()} not row-strided")
    args = ConvGemmArgs()
    args.A, args.a_scale, args.lda, args.Ti, args.To, args.nb = A.data_ptr(), N.ptr(a_scale), _ld(A), Ti, To, nb
    args.in_stride, args.ntaps, args.cin = in_stride, len(offs), cin
    for i, o in enumerate(offs):
        args.off[i] = o
    args.W, args.N, args.K, args.Kp = Wp.data_ptr(), N_, len(offs) * cin, Kp
    args.bias, args.act = N.ptr(bias), act
    args.residual, args.ldr = N.ptr(residual), ldr
    args.c_scale = N.ptr(c_scale)
    args.C, args.ldc, args.To_full, args.out_stride, args.out_off = C.data_ptr(), C.shape[-1], To_full, out_stride, out_off
    args.C_pre = N.ptr(C_pre)
    args.aux, args.ldaux = N.ptr(aux), (aux.shape[-1] if aux is not None else 0)
    args.dropout_p, args.seed = float(dropout_p), N.ptr(seed)
    args.flags = ((GEMM_F_BINARY_SCALE if (binary_scale and a_scale is not None) else 0)
                  | (GEMM_F_A_BF16 if A.dtype == torch.bfloat16 else 0)
                  | (GEMM_F_C_BF16 if C.dtype == torch.bfloat16 else 0)
                  | (GEMM_F_FAST_ACT if (prec == PREC_BF16 and _FAST_ACT) else 0)
                  | (GEMM_F_PRE_BF16 if any(t is not None and t.dtype == torch.bfloat16 for t in (C_pre, aux)) else 0)
                  | (GEMM_F_W_SPLIT if w_split else 0) | (GEMM_F_A_SPLIT if a_split else 0)
                  | (GEMM_F_SPLIT3 if split3 else 0))
    if C_pre is not None and aux is not None and C_pre.dtype != aux.dtype:
        raise ValueError("C_pre and aux must share a dtype")
    log = LAUNCH_LOG
    if log is not None:
        st = torch.cuda.current_stream(C.device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
    lib = N.lib()
    nws = int(lib.mtts_conv_gemm_workspace_size(ctypes.byref(args), prec, tile_cfg, splits))
    ws = torch.empty(nws, dtype=torch.uint8, device=C.device) if nws else None
    N.check(lib.mtts_conv_gemm_ws(ctypes.byref(args), prec, tile_cfg, splits, N.ptr(ws), nws, _stream(C)),
            "mtts_conv_gemm")
    if log is not None:
        e1.record(st)
        M_ = nb * To
        nbytes = (nb * Ti * cin * A.element_size() + (3 if split3 else 2 if w_split else 1) * N_ * Kp * Wp.element_size()
                  + M_ * N_ * C.element_size())
        nbytes += sum(M_ * N_ * t.element_size() for t in (residual, aux, C_pre) if t is not None)
        log.append((e0, e1, 2.0 * M_ * N_ * args.K, prec, nbytes,
                    dict(M=M_, N=N_, K=args.K, cin=cin, ntaps=len(offs), in_stride=in_stride, res=residual is not None,
                         act=act, pre=C_pre is not None, drop=dropout_p > 0, cs=c_scale is not None,
                         asc=a_scale is not None, cfg=tile_cfg, nb=nb, Ti=Ti, To=To, To_full=To_full,
                         out_stride=out_stride, out_off=out_off, offs=list(offs), lda=args.lda, ldc=args.ldc,
                         ldr=ldr, Kp=Kp, prec=prec, flags=int(args.flags), splits=splits, ws=nws,
                         bias=bias is not None, aux=aux is not None)))


# Weight gradients off the critical path: inside side_stream_wgrad() every _wgrad launches on a
# side stream (after the main stream's work so far), so a layer's wgrad + slab reduce overlap the
# dgrad chain that the previous layer waits for -- the backward's kernels are latency-bound and leave
# the chip under-filled one at a time.  Every tensor a side launch touches is kept alive until
# join_side_streams() (the main stream then waits for the side stream), so the caching allocator
# cannot hand its memory to the main stream early; and because that extra reference raises the
# tensors' use count, autograd never accumulates into a pass-through gradient in place while the side
# stream still reads it.  The outputs dw / db are NOT kept (AccumulateGrad then steals them without a
# kernel); nothing on the main stream reads them before the join.  Only for steps where autograd does
# not accumulate into existing .grad tensors (fresh gradients, one micro-batch): the Trainer's graph
# step.
_SIDE_WGRAD = {"on": False, "streams": {}, "keep": []}


@contextlib.contextmanager
def side_stream_wgrad(enabled: bool = True):
    prev = _SIDE_WGRAD["on"]
    _SIDE_WGRAD["on"] = enabled
    try:
        yield
    finally:
        _SIDE_WGRAD["on"] = prev
        join_side_streams()


def join_side_streams():
    for dev, side in _SIDE_WGRAD["streams"].items():
        torch.cuda.current_stream(dev).wait_stream(side)
    _SIDE_WGRAD["keep"].clear()


# Parameter-gradient sums deferred to one batched launch (csrc/reduce.hip): inside
# deferred_grad_sums() the weight-gradient GEMMs and the norm backwards only QUEUE the fixed-order sums
# of their partial slabs; the context exit runs the queue as one launch instead of ~120 small ones.
# The weight-gradient GEMMs themselves are queued too (csrc/conv_gemm.hip, MTTS_DEFER_WGRAD=0 turns it
# off) and a flush launches them batched -- up to 12 layers per launch, each job keeping its own row split,
# so a job's slabs are bitwise those of its own launch with the same plan -- before their sums.  The plan
# itself differs by default (mtts_wgrad_plan_mode(0)): a queued job takes the batched split plan (fewer,
# longer splits), an immediate one the per-launch plan, so the two round differently (both deterministic);
# mtts_wgrad_plan_mode(1) gives every job the batched plan (the tests that compare them bitwise set it).
# The workspaces holding the partials (and the queued GEMMs' inputs) are kept alive until then.  Valid only while nothing reads a
# parameter gradient before the exit: fresh gradients (AccumulateGrad steals them, no copy kernel) of
# LEAF weights -- a Function whose weights are not all leaves (ctx.leaf False) sums at once.
_DEFER = {"on": False, "seam": False, "keep": [], "side_keep": [], "side": {}, "side_used": False,
          # MTTS_SIDE_REDUCE=1 (opt-in): once MTTS_SIDE_REDUCE_JOBS sums are queued, they run on a side
          # stream while the backward continues, joined at the context exit.  Measured slower in the
          # captured step (8.68 -> 9.25..9.39 ms for chunks of 12/24/48 jobs, same box), like the
          # side-stream weight gradients: the default flushes once at the end
          "side_on": os.environ.get("MTTS_SIDE_REDUCE", "0") == "1",
          "chunk": int(os.environ.get("MTTS_SIDE_REDUCE_JOBS", "24")),
          # > 0: flush on the MAIN stream once this many sums are queued (slabs re-read while still in the
          # MALL instead of from HBM at the end of the backward).  0 (default since the weight-gradient GEMMs
          # are queued too): one flush at the end -- the batched launches then hold the whole backward's
          # weight gradients (same box: 8 -> 7.99 ms, 16 7.86, 32 7.77, 64 7.71, 128 7.70, end only 7.64)
          "inline": int(os.environ.get("MTTS_INLINE_REDUCE_JOBS", "0"))}


def _leaves(*ts) -> bool:
    return all(t is None or t.is_leaf for t in ts)


def _keep_partials(*ts):
    if _DEFER["on"]:
        _DEFER["keep"].extend(t for t in ts if t is not None)


@contextlib.contextmanager
def deferred_grad_sums(enabled: bool = True):
    if not enabled or _DEFER["on"]:
        yield
        return
    lib = N.lib()
    lib.mtts_defer_reductions(1)
    _DEFER["on"] = True
    _DEFER["seam"] = False
    ok = False
    try:
        yield
        ok = True
    finally:
        lib.mtts_defer_reductions(0)
        _DEFER["on"] = False
        try:
            if ok:
                N.check(lib.mtts_flush_reductions(torch.cuda.current_stream().cuda_stream), "mtts_flush_reductions")
            else:
                lib.mtts_discard_reductions()
        finally:
            _join_side_sums()
            _DEFER["keep"].clear()  # stream-ordered frees, after the flush launch


def _join_side_sums():
    """The current stream waits for the side-stream sums; their partial slabs may then be freed."""
    if _DEFER["side_used"]:
        main = torch.cuda.current_stream()
        for side in _DEFER["side"].values():
            main.wait_stream(side)
        _DEFER["side_used"] = False
    _DEFER["side_keep"].clear()


def _maybe_side_sums():
    """Inside deferred_grad_sums(): once enough sums are queued, run them on a side stream (after the
    main stream's work so far) while the backward goes on.  Their inputs (partial slabs, kept alive in
    side_keep) and outputs (fresh parameter gradients, which autograd steals without a kernel and
    nothing reads before the join) make this safe."""
    if _DEFER["on"] and not _DEFER["side_on"] and _DEFER["inline"] > 0:
        lib = N.lib()
        if lib.mtts_pending_reductions() >= _DEFER["inline"]:
            N.check(lib.mtts_flush_reductions(torch.cuda.current_stream().cuda_stream), "mtts_flush_reductions")
            _DEFER["keep"].clear()  # stream-ordered frees, after the flush launch
        return
    if _DEFER["on"] and _DEFER["seam"] and _ENC_SIDE_JOBS > 0:
        # past the decoder/encoder seam: the encoder's own queued gradients go to the side stream in chunks
        # (MTTS_ENC_SIDE_JOBS), behind the decoder's batch there, instead of all at the end on the main one
        if N.lib().mtts_pending_reductions() >= _ENC_SIDE_JOBS:
            flush_deferred_side()
        return
    if not (_DEFER["on"] and _DEFER["side_on"]):
        return
    lib = N.lib()
    if lib.mtts_pending_reductions() < _DEFER["chunk"]:
        return
    dev = torch.cuda.current_device()
    side = _DEFER["side"].get(dev)
    if side is None:
        side = _DEFER["side"][dev] = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    N.check(lib.mtts_flush_reductions(side.cuda_stream), "mtts_flush_reductions")
    _DEFER["side_keep"].extend(_DEFER["keep"])
    _DEFER["keep"].clear()
    _DEFER["side_used"] = True


# MTTS_SIDE_FLUSH (default on): at the decoder -> encoder seam of the backward (flow_matching._CfmPack) the
# decoder's queued weight gradients + sums are launched on a side stream, forked there and joined at the
# deferral's exit, so their chip-filling batched launches overlap the text encoder's latency-bound backward
_SIDE_FLUSH = os.environ.get("MTTS_SIDE_FLUSH", "1") != "0"
# MTTS_SIDE_WGRAD_CAP: workgroups the side-flushed weight-gradient batch may occupy (0 = one per block):
# fewer leave CUs to the encoder's backward on the main stream (mtts_wgrad_flush_cap)
_SIDE_CAP = int(os.environ.get("MTTS_SIDE_WGRAD_CAP", "0"))
# MTTS_ENC_SIDE_JOBS > 0: after the seam flush, side-flush again whenever this many sums are queued -- the
# text encoder's own weight gradients then queue behind the decoder's batch on the side stream instead of
# all running on the main one after the encoder's backward (same box: 0 -> 7.20 ms, 8 7.47, 16 7.22,
# 24 7.12, 32 7.10, 40 7.14, 48 7.11, 64 7.11)
_ENC_SIDE_JOBS = int(os.environ.get("MTTS_ENC_SIDE_JOBS", "32"))


def flush_deferred_side() -> None:
    """Inside deferred_grad_sums() (no-op outside, or with MTTS_SIDE_FLUSH=0): everything queued so far
    -- the weight-gradient GEMMs, batched, then the sums -- runs on a side stream forked from the current
    one here, while the backward continues on it; the deferral's exit (or the next main-stream flush)
    joins it.  Inputs and slabs stay alive until then (side_keep); the outputs are fresh parameter
    gradients that nothing reads before the join."""
    if not (_DEFER["on"] and _SIDE_FLUSH) or _DEFER["side_on"]:
        return
    lib = N.lib()
    if lib.mtts_pending_reductions() == 0:
        return
    dev = torch.cuda.current_device()
    side = _DEFER["side"].get(dev)
    if side is None:
        side = _DEFER["side"][dev] = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    lib.mtts_wgrad_flush_cap(_SIDE_CAP)
    try:
        N.check(lib.mtts_flush_reductions(side.cuda_stream), "mtts_flush_reductions")
    finally:
        lib.mtts_wgrad_flush_cap(0)
    _DEFER["side_keep"].extend(_DEFER["keep"])
    _DEFER["keep"].clear()
    _DEFER["side_used"] = True
    _DEFER["seam"] = True


def param_grad_side_stream():
    """Inside deferred_grad_sums() with MTTS_SIDE_FLUSH: the deferral's side stream, already ordered after
    the current stream, for backward work whose only outputs are fresh parameter gradients (joined at the
    deferral's exit like the side flush); None otherwise.  The caller allocates on the current stream and
    hands every tensor the side work reads to keep_for_side()."""
    if not (_DEFER["on"] and _SIDE_FLUSH) or _DEFER["side_on"]:
        return None
    dev = torch.cuda.current_device()
    side = _DEFER["side"].get(dev)
    if side is None:
        side = _DEFER["side"][dev] = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    _DEFER["side_used"] = True
    return side


side_fork = param_grad_side_stream  # the same fork, for forward work that runs ahead (prefetch)


def side_fork_available() -> bool:
    """Whether side_fork() would return a stream (without forking): lets a caller finish the main-stream work
    the side work reads before the fork orders the side stream after it."""
    return bool(_DEFER["on"] and _SIDE_FLUSH) and not _DEFER["side_on"]


def keep_for_side(*ts) -> None:
    _DEFER["side_keep"].extend(t for t in ts if t is not None)


def flush_for_bucket():
    """Inside deferred_grad_sums(), before a data-parallel bucket is packed: every queued weight gradient
    and sum runs now -- on the deferral's side stream when the seam flush is on (the main stream goes on
    with the backward; the seam overlap of the N=1 step is kept), else on the main stream.  Returns the side
    stream whose work so far the packer must wait for (None: everything is ordered on the main stream)."""
    if not _DEFER["on"]:
        return None
    if _SIDE_FLUSH and not _DEFER["side_on"]:
        flush_deferred_side()
        return _DEFER["side"].get(torch.cuda.current_device()) if _DEFER["side_used"] else None
    flush_deferred_grad_sums()
    return None


def flush_deferred_grad_sums() -> None:
    """Runs the queued parameter-gradient sums now (inside deferred_grad_sums(); no-op outside): the
    data-parallel reducer calls it before packing a bucket, so the deferral still batches the sums of
    each bucket into one launch."""
    if not _DEFER["on"]:
        return
    _join_side_sums()
    N.check(N.lib().mtts_flush_reductions(torch.cuda.current_stream().cuda_stream), "mtts_flush_reductions")
    _DEFER["keep"].clear()  # stream-ordered frees, after the flush launch


def _grad_sums(backward):
    """Backward decorator: a Function with non-leaf weights sums its partials at once."""
    @functools.wraps(backward)
    def run(ctx, *grads):
        if not _DEFER["on"]:
            return backward(ctx, *grads)
        if getattr(ctx, "leaf", True):
            out = backward(ctx, *grads)
            _maybe_side_sums()
            return out
        lib = N.lib()
        lib.mtts_defer_reductions(0)
        try:
            return backward(ctx, *grads)
        finally:
            lib.mtts_defer_reductions(1)
    return run


# Data-parallel gradient slots: GradBucketReducer.arm() hands the flat all-reduce buffer's per-parameter views to
# the gradient producers (keyed by the parameter's data pointer), so a weight-gradient kernel writes straight into
# its bucket and the bucket's pack copy has nothing left to move.  A slot is handed out once per
# armed backward: a parameter used twice gets its second gradient in a fresh buffer, which AccumulateGrad adds
# into the slot (the first one, already its .grad) -- the same arithmetic as two fresh buffers.
_GRAD_SLOTS = {"map": None, "used": set()}


def set_grad_slots(mapping) -> None:
    """{parameter data_ptr: fp32 view} for the next backward, or None (fresh gradient buffers)."""
    _GRAD_SLOTS["map"] = mapping
    _GRAD_SLOTS["used"] = set()


def _pkey(t):
    """The slot key of a parameter (its data pointer), None for a non-leaf / absent tensor."""
    return t.data_ptr() if (t is not None and t.is_leaf and t.requires_grad) else None


def _grad_buf(key, shape, device) -> torch.Tensor:
    """The output buffer of one parameter gradient: its armed slot (a flat-buffer view of the same shape), else
    a fresh fp32 tensor."""
    m = _GRAD_SLOTS["map"]
    if m is not None and key is not None and key not in _GRAD_SLOTS["used"]:
        v = m.get(key)
        if v is not None and tuple(v.shape) == tuple(shape):
            _GRAD_SLOTS["used"].add(key)
            # a NEW tensor object on the slot's memory: AccumulateGrad steals a gradient only when nothing else
            # references it -- handed the map's own view it would clone it, on the stream, before the deferred
            # weight-gradient kernels have written it
            return v.view(v.shape)
    return torch.empty(tuple(shape), device=device, dtype=torch.float32)


def _grad_buf_stacked(keys, shapes, rows, K, device):
    """[sum(rows), K] buffer for weights stacked along N (q|k|v): one region of the flat buffer when every
    weight has a slot and the slots lie back to back in stacking order, else a fresh tensor."""
    m = _GRAD_SLOTS["map"]
    if m is not None and all(k is not None and k not in _GRAD_SLOTS["used"] and k in m for k in keys):
        vs = [m[k] for k in keys]
        ok = all(tuple(v.shape) == tuple(sh) for v, sh in zip(vs, shapes))
        off = vs[0].data_ptr()
        for v, r in zip(vs, rows):
            ok = ok and v.data_ptr() == off
            off += r * K * 4
        if ok:
            _GRAD_SLOTS["used"].update(keys)
            return vs[0].as_strided((sum(rows), K), (K, 1))
    return torch.empty(sum(rows), K, device=device, dtype=torch.float32)


def _wgrad(dY, To_full, out_stride, out_off, A, Ti, To, nb, in_stride, offs, cin, N_, dw, strides, *, prec,
           a_scale=None, db=None, rows_per_step=-1, target_blocks=-1, depth=-1):
    if _SIDE_WGRAD["on"] and dY.is_cuda:
        dev = dY.device
        side = _SIDE_WGRAD["streams"].get(dev)
        if side is None:
            side = _SIDE_WGRAD["streams"][dev] = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        # inputs only: an extra reference to dw / db would make AccumulateGrad clone them on the main
        # stream (it steals a gradient only at use count 1) -- reading them before the side stream wrote
        _SIDE_WGRAD["keep"].extend(t for t in (dY, A, a_scale) if t is not None)
        with torch.cuda.stream(side):
            return _wgrad_launch(dY, To_full, out_stride, out_off, A, Ti, To, nb, in_stride, offs, cin, N_, dw,
                                 strides, prec=prec, a_scale=a_scale, db=db, rows_per_step=rows_per_step,
                                 target_blocks=target_blocks, depth=depth)
    return _wgrad_launch(dY, To_full, out_stride, out_off, A, Ti, To, nb, in_stride, offs, cin, N_, dw, strides,
                         prec=prec, a_scale=a_scale, db=db, rows_per_step=rows_per_step,
                         target_blocks=target_blocks, depth=depth)


def _wgrad_launch(dY, To_full, out_stride, out_off, A, Ti, To, nb, in_stride, offs, cin, N_, dw, strides, *, prec,
                  a_scale=None, db=None, rows_per_step=-1, target_blocks=-1, depth=-1):
    args = ConvWgradArgs()
    args.dY, args.ldy, args.To_full, args.out_stride, args.out_off = dY.data_ptr(), _ld(dY), To_full, out_stride, out_off
    args.A, args.a_scale, args.lda, args.Ti, args.To, args.nb = A.data_ptr(), N.ptr(a_scale), _ld(A), Ti, To, nb
    args.in_stride, args.ntaps, args.cin = in_stride, len(offs), cin
    for i, o in enumerate(offs):
        args.off[i] = o
    args.N, args.K = N_, len(offs) * cin
    # every row scale the model passes is a 0/1 sequence mask (as in _gemm)
    args.flags = ((GEMM_F_A_BF16 if A.dtype == torch.bfloat16 else 0) | (GEMM_F_BINARY_SCALE if a_scale is not None else 0)
                  | (WGRAD_F_DY_BF16 if dY.dtype == torch.bfloat16 else 0))
    lib = N.lib()
    ws = torch.empty(int(lib.mtts_conv_wgrad_workspace_size(ctypes.byref(args))), dtype=torch.uint8, device=dY.device)
    # inside deferred_grad_sums() the GEMM itself may be queued (MTTS_DEFER_WGRAD, run batched at the next
    # flush): its inputs stay alive until then, like the slabs
    _keep_partials(ws, dY, A, a_scale)
    log = WGRAD_LOG
    if log is not None:
        st, e0, e1 = _events(dY.device)
    rc = lib.mtts_conv_wgrad_tile(ctypes.byref(args), prec, rows_per_step, target_blocks, depth, dw.data_ptr(), strides[0],
                                  strides[1], strides[2], N.ptr(db), 0, ws.data_ptr(), ws.numel(), _stream(dY))
    N.check(rc, "mtts_conv_wgrad")
    if log is not None:
        e1.record(st)
        M_ = nb * To
        # dY rows read once, the unique A rows once, dW (and db) written once
        nbytes = M_ * N_ * dY.element_size() + nb * Ti * cin * A.element_size() + N_ * args.K * 4
        log.append((e0, e1, 2.0 * M_ * N_ * args.K, prec, nbytes, "wgrad"))


def _check(*ts):
    N.require_device(*[t for t in ts if t is not None])


# ------------------------------------------------------------------------------------------ conv
class _ConvTM(torch.autograd.Function):
    """y[b,u] = (residual + dropout(act(bias + sum_j W_j (x*m)[b, u*stride + j - pad]))) * out_scale
    (nn.Conv1d on x*mask, token-major; act None or ReLU; residual only without act/dropout)."""

    @staticmethod
    def forward(ctx, x, weight, bias, mask, out_scale, stride, padding, act, dropout_p, residual, out_bf16,
                dx_link=None, dx_link_role=None):
        _check(x, weight, mask, residual)
        assert dx_link is None or dx_link_role == "take" or (stride == 1 and dx_link_role == "give")
        ctx.link = (dx_link, dx_link_role)
        assert residual is None or (act == ACT_NONE and dropout_p == 0.0)
        prec = gemm_precision()
        x = _actc(x, prec)
        B, Ti, Cin = x.shape
        Cout, _, k = weight.shape
        if x.dtype == torch.bfloat16 and not _bf16_operand_ok(Cin):
            x = x.float()
        To = (Ti + 2 * padding - k) // stride + 1
        Wp, Kp = packed(spec_conv_fwd(weight), prec)
        # the backward's dgrad operands come from the same packing pass (weight_pack_scope)
        ctx.wd = None
        if ctx.needs_input_grad[0]:
            ctx.wd = [packed(spec_conv_dgrad(weight), prec)] if stride == 1 else \
                [packed(spec_conv_dgrad(weight, (ph + padding) % stride, stride), prec)
                 if len(range((ph + padding) % stride, k, stride)) else None for ph in range(stride)]
        # bf16 output (bf16-mixed, out_bf16): GroupNorm input / next GEMM operand; its gradient then comes
        # back as bf16 too, and is the dgrad GEMM's bf16 A operand
        y16 = out_bf16 and prec == PREC_BF16 and _bf16_operand_ok(Cout) and act == ACT_NONE and dropout_p == 0.0
        y = torch.empty(B, To, Cout, device=x.device, dtype=torch.bfloat16 if y16 else torch.float32)
        mask = _f32c(mask)
        out_scale = _f32c(out_scale)
        bias_c = _f32c(bias)
        seed = _new_seed(x.device) if dropout_p > 0 else None
        _gemm(x, Ti, To, B, stride, [j - padding for j in range(k)], Cin, Wp, Kp, Cout, y, To, prec=prec,
              a_scale=mask, bias=bias_c, c_scale=out_scale, act=act, dropout_p=dropout_p, seed=seed,
              residual=_f32c(residual))
        ctx.save_for_backward(x, weight, mask, out_scale, y if act != ACT_NONE else None)
        ctx.leaf = _leaves(weight, bias)
        ctx.keys = (_pkey(weight), _pkey(bias))
        ctx.cfg = (stride, padding, prec, bias is not None, act, dropout_p, seed, residual is not None)
        return y

    @staticmethod
    @_grad_sums
    def backward(ctx, dy):
        x, weight, mask, out_scale, y = ctx.saved_tensors
        stride, pad, prec, has_bias, act, p, seed, has_res = ctx.cfg
        dy = _actc(dy, prec)
        if dy.dtype == torch.bfloat16 and (out_scale is not None or act != ACT_NONE or p > 0
                                           or not _bf16_operand_ok(dy.shape[-1])):
            dy = dy.float()
        if out_scale is not None:
            dy = dy * out_scale.unsqueeze(-1)
        dres = dy if has_res else None
        if act != ACT_NONE or p > 0:  # through the epilogue ReLU / dropout (gate from the output y)
            g = torch.empty_like(dy)
            N.check(N.lib().mtts_act_dropout_bwd(dy.data_ptr(), N.ptr(y), g.data_ptr(), dy.shape[0] * dy.shape[1],
                                                 dy.shape[2], dy.shape[2], act, float(p), N.ptr(seed), _stream(g)),
                    "mtts_act_dropout_bwd")
            dy = g
        B, Ti, Cin = x.shape
        Cout, _, k = weight.shape
        To = dy.shape[1]
        dx = dw = db = None
        link, role = ctx.link
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)  # in x's storage: a bf16 x (a GroupNorm output) gets a bf16 gradient
            # GradLink "take": the other consumer's gradient of the same x (already computed: its backward
            # ran first) is added in this dgrad's epilogue -- the autograd sum of the two input gradients
            # without its add kernel.  (acc + other) * m equals m * acc + other: m is 0/1 and other is
            # either m-scaled (a conv's dgrad) or zero wherever m is (the masked decoder rows).  A row-strided
            # fp32 view (a slice of the up path's concat gradient) is read in place.
            other = link.pop() if role == "take" else None
            fuse = (other is not None and other.dtype == dx.dtype == torch.float32 and other.stride(-1) == 1
                    and other.shape == dx.shape and other.stride(0) == other.shape[1] * other.stride(1))
            if stride == 1:
                Wd, Kp = ctx.wd[0]
                _gemm(dy, To, Ti, B, 1, [pad - j for j in range(k)], Cout, Wd, Kp, Cin, dx, Ti, prec=prec,
                      c_scale=mask, residual=other if fuse else None)
            else:  # stride-2 dgrad = transposed conv = one GEMM per output phase
                for ph in range(stride):
                    j0 = (ph + pad) % stride  # taps of this phase: j0, j0+stride, ... (a slice: no
                    js = list(range(j0, k, stride))  # host->device index copy, legal in graph capture)
                    nrows = (Ti - ph + stride - 1) // stride
                    if not js or nrows <= 0:
                        dx[:, ph::stride].zero_()
                        continue
                    Wd, Kp = ctx.wd[ph]
                    _gemm(dy, To, nrows, B, 1, [(ph + pad - j) // stride for j in js], Cout, Wd, Kp, Cin, dx, Ti,
                          stride, ph, prec=prec, c_scale=mask, residual=other if fuse else None)
            if other is not None and not fuse:  # bf16 x or an unusual layout: autograd's sum, done here
                dx = dx + other
        if ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2]):
            dw = _grad_buf(ctx.keys[0], weight.shape, x.device)
            db = _grad_buf(ctx.keys[1], (Cout,), x.device) if has_bias else None
            _wgrad(dy, To, 1, 0, x, Ti, To, B, stride, [j - pad for j in range(k)], Cin, Cout, dw,
                   (Cin * k, k, 1), prec=prec, a_scale=mask, db=db)
        if role == "give" and dx is not None:  # handed to the "take" conv of the same x (GradLink)
            link.put(dx)
            dx = None
        return dx, dw, db, None, None, None, None, None, None, dres, None, None, None


class _ConvTransposeTM(torch.autograd.Function):
    """ConvTranspose1d(k, stride 2, padding p) of x*mask (Upsample1D, decoder.py:112): two phase GEMMs."""

    @staticmethod
    def forward(ctx, x, weight, bias, mask):
        _check(x, weight, mask)
        prec = gemm_precision()
        x = _f32c(x)
        mask = _f32c(mask)
        B, T, Cin = x.shape
        _, Cout, k = weight.shape
        pad, s = 1, 2
        To_full = (T - 1) * s - 2 * pad + k
        y = torch.empty(B, To_full, Cout, device=x.device, dtype=torch.float32)
        bias_c = _f32c(bias)
        for ph in range(s):
            j0 = (ph + pad) % s  # taps of this phase: j0, j0+s, ... (slice, not a host index list)
            js = list(range(j0, k, s))
            nrows = (To_full - ph + s - 1) // s
            Wp, Kp = packed(spec_convT_fwd(weight, j0, s), prec)
            _gemm(x, T, nrows, B, 1, [(ph + pad - j) // s for j in js], Cin, Wp, Kp, Cout, y, To_full, s, ph,
                  prec=prec, a_scale=mask, bias=bias_c)
        ctx.wd = packed(spec_convT_dgrad(weight), prec) if ctx.needs_input_grad[0] else None
        ctx.save_for_backward(x, weight, mask)
        ctx.leaf = _leaves(weight, bias)
        ctx.keys = (_pkey(weight), _pkey(bias))
        ctx.cfg = (prec, bias is not None)
        return y

    @staticmethod
    @_grad_sums
    def backward(ctx, dy):
        x, weight, mask = ctx.saved_tensors
        prec, has_bias = ctx.cfg
        # the up path hands a channel slice of its concat gradient: read in place (row-strided operand)
        dy = dy if _row_strided_f32(dy) else _f32c(dy)
        B, T, Cin = x.shape
        _, Cout, k = weight.shape
        pad, s = 1, 2
        T2 = dy.shape[1]
        dx = dw = db = None
        offs = [j - pad for j in range(k)]
        if ctx.needs_input_grad[0]:  # dgrad of a transposed conv = stride-2 conv over dy
            dx = torch.empty_like(x)
            Wd, Kp = ctx.wd
            _gemm(dy, T2, T, B, s, offs, Cout, Wd, Kp, Cin, dx, T, prec=prec, c_scale=mask)
        if ctx.needs_input_grad[1]:
            xm = x * mask.unsqueeze(-1) if mask is not None else x
            dw = _grad_buf(ctx.keys[0], weight.shape, x.device)
            # dW[c, n, j] = sum_s xm[s, c] dy[2s + j - pad, n]
            _wgrad(xm, T, 1, 0, dy, T2, T, B, s, offs, Cout, Cin, dw,
                   (weight.stride(0), weight.stride(1), weight.stride(2)), prec=prec)
        if has_bias and ctx.needs_input_grad[2]:
            # column sums of dy (rows may be strided: a slice of the concat gradient) in a fixed order:
            # 128-row partials + a job in the step's batched gradient sums (torch's reduction: 26 us)
            db = _grad_buf(ctx.keys[1], (Cout,), dy.device)
            rows = B * T2
            ws = torch.empty(int(N.lib().mtts_colsum_workspace_size(rows, Cout)) // 4, device=dy.device,
                             dtype=torch.float32)
            _keep_partials(ws, dy)
            N.check(N.lib().mtts_colsum(dy.data_ptr(), rows, Cout, _ld(dy), db.data_ptr(), 0, ws.data_ptr(),
                                        ws.numel() * 4, _stream(dy)), "mtts_colsum")
        return dx, dw, db, None


class _LinearTM(torch.autograd.Function):
    """x @ W^T + b -> dropout -> + residual  (diffusers to_q/k/v/to_out Linear + Dropout).  W may be
    several weights stacked along N (the fused q|k|v projection), each receiving its own gradient."""

    @staticmethod
    def forward(ctx, x, bias, residual, dropout_p, in_scale, out_scale, link, *weights):
        _check(x, residual, in_scale, out_scale, *weights)
        prec = gemm_precision()
        ctx.link = link  # (GradLink, "take" | "give_res") or None
        shp = x.shape
        x2 = _f32c(x).reshape(-1, shp[-1])
        M, K = x2.shape
        Nout = sum(w.shape[0] for w in weights)
        assert all(w.dim() == 2 or (w.dim() == 3 and w.shape[2] == 1) for w in weights)
        Wp, Kp = packed(spec_linear(weights), prec)
        ctx.wd = packed(spec_linear(weights, dgrad=True), prec) if ctx.needs_input_grad[0] else None
        y = torch.empty(M, Nout, device=x.device, dtype=torch.float32)
        res2 = _f32c(residual).reshape(M, Nout) if residual is not None else None
        seed = _new_seed(x.device) if dropout_p > 0 else None
        ins = _f32c(in_scale).reshape(M) if in_scale is not None else None
        outs = _f32c(out_scale).reshape(M) if out_scale is not None else None
        _gemm(x2, M, M, 1, 1, [0], K, Wp, Kp, Nout, y, M, prec=prec, bias=_f32c(bias), residual=res2,
              dropout_p=dropout_p, seed=seed, a_scale=ins, c_scale=outs)
        ctx.save_for_backward(x2, ins, outs)
        ctx.leaf = _leaves(bias, *weights)
        ctx.keys = (_pkey(bias), [_pkey(w) for w in weights])
        ctx.cfg = (prec, bias is not None, residual is not None, shp, dropout_p, seed,
                   [w.shape[0] for w in weights], K)
        ctx.wshapes = [w.shape for w in weights]
        return y.reshape(*shp[:-1], Nout)

    @staticmethod
    @_grad_sums
    def backward(ctx, dy):
        x2, ins, outs = ctx.saved_tensors
        prec, has_bias, has_res, shp, p, seed, rows, K = ctx.cfg
        Nout = sum(rows)
        dy2 = _f32c(dy).reshape(-1, Nout)
        M = dy2.shape[0]
        if outs is not None:  # y = (residual + z) * out_scale
            dy2 = dy2 * outs.unsqueeze(-1)
        dres = dy2.reshape(dy.shape) if has_res else None
        if p > 0:  # gradient through the epilogue dropout: regenerate the forward's mask
            g = torch.empty_like(dy2)
            N.check(N.lib().mtts_dropout_apply(dy2.data_ptr(), g.data_ptr(), M, Nout, Nout, float(p),
                                               seed.data_ptr(), _stream(g)), "mtts_dropout_apply")
            dy2 = g
        dx = db = None
        dws = [None] * len(rows)
        Np = _r8(Nout)
        if Np != Nout:  # narrow outputs (the duration predictor's 1-channel projection): zero-pad dy to 8
            dyp = torch.zeros(M, Np, device=dy2.device, dtype=torch.float32)  # columns; W^T is packed with
            dyp[:, :Nout] = dy2  # zero columns to Np already, so dgrad is exact; dW/db keep rows < Nout
            dy2 = dyp
        link, role = ctx.link if ctx.link is not None else (None, None)
        if role == "give_res" and dres is not None:  # the residual's gradient goes to the taker's dgrad
            link.put(dres)
            dres = None
        if ctx.needs_input_grad[0]:
            Wd, Kp = ctx.wd
            dx = torch.empty(M, K, device=dy2.device, dtype=torch.float32)
            # "take": + the other consumer's gradient of x, (acc + other) * in_scale -- equal to autograd's
            # sum when `other` vanishes wherever in_scale does (the caller's guarantee, see GradLink users)
            other = link.pop() if role == "take" else None
            fuse = other is not None and other.dtype == torch.float32 and other.is_contiguous() and other.numel() == M * K
            _gemm(dy2, M, M, 1, 1, [0], Np, Wd, Kp, K, dx, M, prec=prec, c_scale=ins,
                  residual=other.view(M, K) if fuse else None)
            dx = dx.reshape(*shp)
            if other is not None and not fuse:
                dx = dx + other
        if any(ctx.needs_input_grad[6:]) or (has_bias and ctx.needs_input_grad[1]):
            bkey, wkeys = ctx.keys
            dw = _grad_buf_stacked(wkeys, ctx.wshapes, rows, K, dy2.device) if Np == Nout else \
                torch.empty(Np, K, device=dy2.device, dtype=torch.float32)
            db = (_grad_buf(bkey, (Np,), dy2.device) if Np == Nout else
                  torch.empty(Np, device=dy2.device, dtype=torch.float32)) if has_bias else None
            _wgrad(dy2, M, 1, 0, x2, M, M, 1, 1, [0], K, Np, dw, (K, 1, 0), prec=prec, db=db, a_scale=ins)
            dws = [d.view(w_shape) for d, w_shape in zip(dw[:Nout].split(rows, dim=0), ctx.wshapes)]
            db = db[:Nout] if db is not None else None
        return (dx, db, dres, None, None, None, None, *dws)


class _FeedForwardTM(torch.autograd.Function):
    """residual + dropout(gelu(x W1^T + b1)) W2^T + b2   (diffusers GELU -> Dropout -> Linear,
    transformer.py:155-188).  The pre-activation is stored by the first GEMM's epilogue; the backward
    folds GELU' and the regenerated dropout mask into the second GEMM's dgrad epilogue."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, residual, dropout_p):
        _check(x, w1, w2, residual)
        prec = gemm_precision()
        shp = x.shape
        x2 = _f32c(x).reshape(-1, shp[-1])
        M, K = x2.shape
        H, Nout = w1.shape[0], w2.shape[0]
        W1p, K1p = packed(spec_linear((w1,)), prec)
        W2p, K2p = packed(spec_linear((w2,)), prec)
        ctx.w2t = packed(spec_linear((w2,), dgrad=True), prec) if any(ctx.needs_input_grad) else None
        ctx.w1t = packed(spec_linear((w1,), dgrad=True), prec) if ctx.needs_input_grad[0] else None
        # bf16-mixed: the GELU output is only ever the next GEMM's (and its wgrad's) bf16 MFMA operand,
        # so it is stored as bf16 -- half the bytes written here and read twice later; the saved
        # pre-activation (read once, by GELU' in the backward) too, as autocast would keep it
        h16 = prec == PREC_BF16 and os.environ.get("MTTS_FF_FP32_HIDDEN") != "1"
        z16 = prec == PREC_BF16 and os.environ.get("MTTS_FF_FP32_PRE") != "1"
        z = torch.empty(M, H, device=x.device, dtype=torch.bfloat16 if z16 else torch.float32)
        h = torch.empty(M, H, device=x.device, dtype=torch.bfloat16 if h16 else torch.float32)
        seed = _new_seed(x.device) if dropout_p > 0 else None
        _gemm(x2, M, M, 1, 1, [0], K, W1p, K1p, H, h, M, prec=prec, bias=_f32c(b1), act=ACT_GELU, C_pre=z,
              dropout_p=dropout_p, seed=seed)
        y = torch.empty(M, Nout, device=x.device, dtype=torch.float32)
        res2 = _f32c(residual).reshape(M, Nout) if residual is not None else None
        _gemm(h, M, M, 1, 1, [0], H, W2p, K2p, Nout, y, M, prec=prec, bias=_f32c(b2), residual=res2)
        ctx.save_for_backward(x2, z, h, w1, w2)
        ctx.leaf = _leaves(w1, b1, w2, b2)
        ctx.keys = (_pkey(w1), _pkey(b1), _pkey(w2), _pkey(b2))
        ctx.cfg = (prec, shp, residual is not None, dropout_p, seed, b1 is not None, b2 is not None)
        return y.reshape(*shp[:-1], Nout)

    @staticmethod
    @_grad_sums
    def backward(ctx, dy):
        x2, z, h, w1, w2 = ctx.saved_tensors
        prec, shp, has_res, p, seed, has_b1, has_b2 = ctx.cfg
        H, K = w1.shape
        Nout = w2.shape[0]
        dy2 = _f32c(dy).reshape(-1, Nout)
        M = dy2.shape[0]
        dev = dy2.device
        kw1, kb1, kw2, kb2 = ctx.keys
        dw2 = _grad_buf(kw2, w2.shape, dev)
        db2 = _grad_buf(kb2 if has_b2 else None, (Nout,), dev)
        _wgrad(dy2, M, 1, 0, h, M, M, 1, 1, [0], H, Nout, dw2, (H, 1, 0), prec=prec, db=db2)
        W2t, K2p = ctx.w2t
        dz = torch.empty(M, H, device=dev, dtype=torch.float32)
        _gemm(dy2, M, M, 1, 1, [0], Nout, W2t, K2p, H, dz, M, prec=prec, act=ACT_DGELU, aux=z, dropout_p=p,
              seed=seed)
        dw1 = _grad_buf(kw1, w1.shape, dev)
        db1 = _grad_buf(kb1 if has_b1 else None, (H,), dev)
        _wgrad(dz, M, 1, 0, x2, M, M, 1, 1, [0], K, H, dw1, (K, 1, 0), prec=prec, db=db1)
        dx = None
        if ctx.needs_input_grad[0]:
            W1t, K1p = ctx.w1t
            dx = torch.empty(M, K, device=dev, dtype=torch.float32)
            _gemm(dz, M, M, 1, 1, [0], H, W1t, K1p, K, dx, M, prec=prec)
            dx = dx.reshape(*shp)
        return (dx, dw1, db1 if has_b1 else None, dw2, db2 if has_b2 else None, (dy if has_res else None),
                None)


class _ConvFFNTM(torch.autograd.Function):
    """The text encoder's FFN + residual (text_encoder.py:235-253, 307-313), token-major:
        h = dropout_in(relu(conv1(x * m)))              (epilogue ReLU + dropout, h stored)
        y = (residual + dropout_out(conv2(h))) * m       (epilogue dropout, residual, row mask)
    The reference masks only the FFN's input and output (conv_net(x * x_mask) * x_mask): conv2 reads
    the UNMASKED h, so rows next to the padding see the padded rows' relu(bias + leakage).
    dropout_out is the FFN's own Dropout followed by the Encoder's self.dropout: two independent
    Bernoulli(1-p) masks are one Bernoulli((1-p)^2) mask with scale 1/(1-p)^2 -- same distribution.
    Backward: regenerated masks; ReLU' folded into conv2's dgrad epilogue (gate = h > 0)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, mask, residual, p_in, p_out):
        _check(x, w1, w2, mask, residual)
        prec = gemm_precision()
        # the encoder's residual IS the FFN input: the backward adds the residual gradient in the input
        # dgrad's epilogue (one tensor, no autograd accumulate kernel)
        ctx.res_is_x = residual is x
        x = _f32c(x)
        B, T, Cin = x.shape
        F_, _, k = w1.shape
        Cout = w2.shape[0]
        pad = k // 2
        offs = [j - pad for j in range(k)]
        m = _f32c(mask)
        W1p, K1p = packed(spec_conv_fwd(w1), prec)
        W2p, K2p = packed(spec_conv_fwd(w2), prec)
        ctx.w2d = packed(spec_conv_dgrad(w2), prec) if any(ctx.needs_input_grad) else None
        ctx.w1d = packed(spec_conv_dgrad(w1), prec) if ctx.needs_input_grad[0] else None
        s1 = _new_seed(x.device) if p_in > 0 else None
        s2 = _new_seed(x.device) if p_out > 0 else None
        h = torch.empty(B, T, F_, device=x.device, dtype=torch.float32)
        _gemm(x, T, T, B, 1, offs, Cin, W1p, K1p, F_, h, T, prec=prec, a_scale=m, bias=_f32c(b1), act=ACT_RELU,
              dropout_p=p_in, seed=s1)
        y = torch.empty(B, T, Cout, device=x.device, dtype=torch.float32)
        _gemm(h, T, T, B, 1, offs, F_, W2p, K2p, Cout, y, T, prec=prec, bias=_f32c(b2), dropout_p=p_out,
              seed=s2, residual=_f32c(residual), c_scale=m)
        ctx.save_for_backward(x, h, m)
        ctx.leaf = _leaves(w1, b1, w2, b2)
        ctx.keys = (_pkey(w1), _pkey(b1), _pkey(w2), _pkey(b2))
        ctx.cfg = (prec, k, p_in, p_out, s1, s2, residual is not None, w1.shape, w2.shape)
        return y

    @staticmethod
    @_grad_sums
    def backward(ctx, dy):
        x, h, m = ctx.saved_tensors
        prec, k, p_in, p_out, s1, s2, has_res, w1s, w2s = ctx.cfg
        B, T, Cin = x.shape
        F_, Cout = w1s[0], w2s[0]
        pad = k // 2
        offs = [j - pad for j in range(k)]
        doffs = [pad - j for j in range(k)]
        fuse = ctx.res_is_x and has_res and ctx.needs_input_grad[0]
        if fuse and p_out > 0:
            # the masked output's gradient g = dy * m is only read by the dropout backward (which applies
            # the row mask itself) and as the residual of the input dgrad, where (acc + dy) * m equals
            # (acc + dy * m) * m for a 0/1 mask: dy is used as is, g never materialised
            g = _f32c(dy)
            dz2 = torch.empty_like(g)
            N.check(N.lib().mtts_act_dropout_bwd_scaled(g.data_ptr(), None, m.data_ptr(), dz2.data_ptr(), B * T, Cout,
                                                        Cout, ACT_NONE, float(p_out), s2.data_ptr(), _stream(g)),
                    "mtts_act_dropout_bwd_scaled")
        else:
            g = _f32c(dy) * m.unsqueeze(-1)
            dz2 = g
            if p_out > 0:
                dz2 = torch.empty_like(g)
                N.check(N.lib().mtts_act_dropout_bwd(g.data_ptr(), None, dz2.data_ptr(), B * T, Cout, Cout, ACT_NONE,
                                                     float(p_out), s2.data_ptr(), _stream(g)), "mtts_act_dropout_bwd")
        dres = g if has_res else None
        kw1, kb1, kw2, kb2 = ctx.keys
        dw2 = _grad_buf(kw2, w2s, x.device)
        db2 = _grad_buf(kb2, (Cout,), x.device)
        _wgrad(dz2, T, 1, 0, h, T, T, B, 1, offs, F_, Cout, dw2, (F_ * k, k, 1), prec=prec, db=db2)
        W2d, K2d = ctx.w2d
        dz1 = torch.empty_like(h)  # d(conv1 pre-activation) = dgrad * [h > 0] * keep_in / (1 - p_in)
        _gemm(dz2, T, T, B, 1, doffs, Cout, W2d, K2d, F_, dz1, T, prec=prec, act=ACT_DRELU, aux=h,
              dropout_p=p_in, seed=s1)
        dw1 = _grad_buf(kw1, w1s, x.device)
        db1 = _grad_buf(kb1, (F_,), x.device)
        _wgrad(dz1, T, 1, 0, x, T, T, B, 1, offs, Cin, F_, dw1, (Cin * k, k, 1), prec=prec, a_scale=m, db=db1)
        dx = None
        if ctx.needs_input_grad[0]:
            W1d, K1d = ctx.w1d
            dx = torch.empty_like(x)
            # (dgrad + g) * m = dgrad * m + g: g = dy * m already vanishes on the masked rows
            _gemm(dz1, T, T, B, 1, doffs, F_, W1d, K1d, Cin, dx, T, prec=prec, c_scale=m,
                  residual=g if fuse else None)
            if fuse:
                dres = None
        return dx, dw1, db1, dw2, db2, None, dres, None, None


def conv_ffn_tm(x, w1, b1, w2, b2, mask, residual=None, p_in: float = 0.0, p_out: float = 0.0):
    """(residual + dropout_out(conv2(dropout_in(relu(conv1(x*m)))))) * m, token-major (text encoder
    FFN, text_encoder.py:235-253); conv weights [F, Cin, k] / [Cout, F, k], odd k <= 8."""
    return _ConvFFNTM.apply(x, w1, b1, w2, b2, mask, residual, float(p_in), float(p_out))


# ------------------------------------------------------------------------------------------ norms
class _GroupNormMishTM(torch.autograd.Function):
    """mish(GN(h)) * mask + add; in bf16-mixed mode h may be bf16 (a conv GEMM's bf16 output) and y is
    written as bf16 when asked (it only feeds the next conv's GEMM); dh comes back in h's storage."""

    @staticmethod
    def forward(ctx, h, gamma, beta, mask, add, groups, eps, out_bf16):
        _check(h, gamma, mask, add)
        prec = gemm_precision()
        h = _actc(h, prec)
        B, T, C = h.shape
        y16 = out_bf16 and prec == PREC_BF16
        y = torch.empty(B, T, C, device=h.device, dtype=torch.bfloat16 if y16 else torch.float32)
        mean = torch.empty(B, groups, device=h.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        gamma_c, beta_c, mask_c, add_c = _f32c(gamma), _f32c(beta), _f32c(mask), _f32c(add)
        flags = (NORM_F_X_BF16 if h.dtype == torch.bfloat16 else 0) | (NORM_F_Y_BF16 if y16 else 0)
        N.check(N.lib().mtts_gn_mish_fwd_ex(h.data_ptr(), gamma_c.data_ptr(), beta_c.data_ptr(), N.ptr(mask_c),
                                            N.ptr(add_c), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(), B, T, C,
                                            groups, float(eps), flags, _stream(h)), "mtts_gn_mish_fwd")
        ctx.save_for_backward(h, gamma_c, beta_c, mask_c, mean, rstd)
        ctx.leaf = _leaves(gamma, beta)
        ctx.keys = (_pkey(gamma), _pkey(beta))
        ctx.cfg = (groups, add is not None)
        return y

    @staticmethod
    @_grad_sums
    def backward(ctx, dy):
        h, gamma, beta, mask, mean, rstd = ctx.saved_tensors
        groups, has_add = ctx.cfg
        h16 = h.dtype == torch.bfloat16
        dy = dy.contiguous() if (h16 and dy.dtype == torch.bfloat16) else _f32c(dy)
        B, T, C = h.shape
        dh = torch.empty_like(h)
        dg = _grad_buf(ctx.keys[0], (C,), h.device)
        dbt = _grad_buf(ctx.keys[1], (C,), h.device)
        dadd = torch.empty(B, C, device=h.device, dtype=torch.float32) if has_add else None
        flags = (NORM_F_X_BF16 | NORM_F_Y_BF16 if h16 else 0) | (NORM_F_DY_BF16 if dy.dtype == torch.bfloat16 else 0)
        lib = N.lib()
        ws = torch.empty(int(lib.mtts_gn_mish_bwd_workspace_size(B, C)), dtype=torch.uint8, device=h.device)
        _keep_partials(ws)
        N.check(lib.mtts_gn_mish_bwd_ex(dy.data_ptr(), h.data_ptr(), gamma.data_ptr(), beta.data_ptr(), N.ptr(mask),
                                        mean.data_ptr(), rstd.data_ptr(), dh.data_ptr(), dg.data_ptr(), dbt.data_ptr(),
                                        N.ptr(dadd), B, T, C, groups, flags, ws.data_ptr(), ws.numel(), _stream(h)),
                "mtts_gn_mish_bwd")
        return dh, dg, dbt, None, dadd, None, None, None


class _LayerNormTM(torch.autograd.Function):
    """LayerNorm over the last dim, optionally followed by a fused ReLU and/or dropout (the text
    encoder's LN -> ReLU -> Dropout and LN -> Dropout, text_encoder.py:48-55, 81-95)."""

    @staticmethod
    def forward(ctx, x, w, b, eps, act, dropout_p):
        _check(x, w)
        shp = x.shape
        x2 = _f32c(x).reshape(-1, shp[-1])
        M, C = x2.shape
        y = torch.empty_like(x2)
        mean = torch.empty(M, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        w_c, b_c = _f32c(w), _f32c(b)
        seed = _new_seed(x.device) if dropout_p > 0 else None
        N.check(N.lib().mtts_layernorm_fwd(x2.data_ptr(), w_c.data_ptr(), b_c.data_ptr(), y.data_ptr(),
                                           mean.data_ptr(), rstd.data_ptr(), M, C, float(eps), act, float(dropout_p),
                                           N.ptr(seed), _stream(x2)), "mtts_layernorm_fwd")
        ctx.save_for_backward(x2, w_c, b_c, mean, rstd)
        ctx.leaf = _leaves(w, b)
        ctx.keys = (_pkey(w), _pkey(b))
        ctx.cfg = (shp, act, float(dropout_p), seed)
        return y.reshape(shp)

    @staticmethod
    @_grad_sums
    def backward(ctx, dy):
        x2, w, b, mean, rstd = ctx.saved_tensors
        shp, act, p, seed = ctx.cfg
        M, C = x2.shape
        dy2 = _f32c(dy).reshape(M, C)
        dx = torch.empty_like(x2)
        dw = _grad_buf(ctx.keys[0], (C,), x2.device)
        db = _grad_buf(ctx.keys[1], (C,), x2.device)
        lib = N.lib()
        ws = torch.empty(max(int(lib.mtts_layernorm_bwd_workspace_size(M, C)), 1), dtype=torch.uint8,
                         device=x2.device)
        _keep_partials(ws)
        N.check(lib.mtts_layernorm_bwd(dy2.data_ptr(), x2.data_ptr(), w.data_ptr(), b.data_ptr(), mean.data_ptr(),
                                       rstd.data_ptr(), dx.data_ptr(), dw.data_ptr(), db.data_ptr(), M, C, act, p,
                                       N.ptr(seed), ws.data_ptr(), ws.numel(), _stream(x2)), "mtts_layernorm_bwd")
        return dx.reshape(shp), dw, db, None, None, None


# ------------------------------------------------------------------------------------------ public ops
class GradLink:
    """Two stride-1 convs reading the same x (Resnet1D's block1 conv and res_conv, decoder.py:83-86):
    the one that runs LATER in the forward ("give") hands its input gradient to the earlier one
    ("take") instead of returning it, and the taker adds it in its dgrad GEMM epilogue -- one GEMM
    output instead of two plus autograd's add.  Autograd runs the giver's backward first because the
    taker's output gradient depends on it (the giver's residual input is computed from the taker's
    output).  If the giver never ran (no input gradient), the taker adds nothing."""

    __slots__ = ("buf",)

    def __init__(self):
        self.buf = None

    def put(self, t):
        assert self.buf is None, "GradLink: two gradients handed over"
        self.buf = t

    def pop(self):
        t, self.buf = self.buf, None
        return t


class _CatSkipTM(torch.autograd.Function):
    """[h | skip] on channels (the up path's einops pack, decoder.py:341).  Backward: h's gradient is the
    first channel slice; skip's slice goes to the skip's earlier consumer through a GradLink (that conv
    adds it in its dgrad epilogue, reading the slice in place) instead of autograd's strided add."""

    @staticmethod
    def forward(ctx, h, skip, link):
        ctx.c1, ctx.link = h.shape[-1], link
        return torch.cat([h, skip], dim=-1)

    @staticmethod
    def backward(ctx, d):
        d1, d2 = d[..., : ctx.c1], d[..., ctx.c1:]
        if ctx.link is not None:
            ctx.link.put(d2)
            d2 = None
        return d1, d2, None


def cat_skip_tm(h, skip, link: "GradLink | None" = None):
    return _CatSkipTM.apply(h, skip, link)


def conv_tm(x, weight, bias, mask=None, stride: int = 1, padding: int | None = None, out_scale=None,
            relu: bool = False, dropout_p: float = 0.0, residual=None, out_bf16: bool = False,
            dx_link: GradLink | None = None, dx_link_role: str | None = None):
    """y = (residual + dropout(relu(Conv1d(x * mask)))) * out_scale, token-major.  x [B,T,Cin], weight
    [Cout,Cin,k] (nn.Conv1d layout, k <= 8), mask/out_scale [B,T] or None.  dx_link / dx_link_role
    ("take" / "give"): see GradLink.
    decoder.py:59,65,78,85,95,192,239,248,251,369-371; text_encoder.py:48-57, 81-96."""
    if padding is None:
        padding = weight.shape[-1] // 2
    return _ConvTM.apply(x, weight, bias, mask, out_scale, stride, padding, ACT_RELU if relu else ACT_NONE,
                         float(dropout_p), residual, bool(out_bf16), dx_link, dx_link_role)


def conv_transpose_tm(x, weight, bias, mask=None):
    """ConvTranspose1d(k=4, s=2, p=1) of x * mask; weight [Cin,Cout,4].  decoder.py:112-116."""
    return _ConvTransposeTM.apply(x, weight, bias, mask)


def group_norm_mish_tm(h, gamma, beta, groups: int, mask=None, add=None, eps: float = 1e-5, out_bf16: bool = False):
    """mish(GroupNorm(h)) * mask (+ add[b, c]): Block1D tail (decoder.py:58-66) with Resnet1D's
    time-embedding add (decoder.py:82-83) fused; statistics over the full padded length.  out_bf16: in
    bf16-mixed mode, store the result as bf16 (when its only consumer is a conv GEMM)."""
    return _GroupNormMishTM.apply(h, gamma, beta, mask, add, groups, eps, bool(out_bf16))


def layer_norm_tm(h, weight, bias, eps: float = 1e-5, relu: bool = False, dropout_p: float = 0.0):
    """LayerNorm over the last dim [-> ReLU] [-> dropout(p)], one kernel each way."""
    return _LayerNormTM.apply(h, weight, bias, eps, ACT_RELU if relu else ACT_NONE, float(dropout_p))


def linear_tm(x, weight, bias=None, residual=None, dropout_p: float = 0.0, in_scale=None, out_scale=None,
              dx_link: GradLink | None = None, dx_link_role: str | None = None):
    """(residual + dropout((x * in_scale) @ W^T + b)) * out_scale   (diffusers Linear [+ Dropout]
    [+ residual]; the text encoder's masked 1x1 convs).  `weight` may be a tuple of weights stacked along
    the output dim (one GEMM, one gradient per weight); a weight may be an nn.Conv1d weight [N, K, 1].
    in_scale / out_scale: per-row [B, T] (or [M]) scales, e.g. the sequence mask.
    dx_link / dx_link_role: "take" adds the linked gradient into dx's dgrad epilogue; "give_res" hands the
    residual's gradient to it (GradLink)."""
    ws = tuple(weight) if isinstance(weight, (tuple, list)) else (weight,)
    link = (dx_link, dx_link_role) if dx_link is not None else None
    assert link is None or dx_link_role in ("take", "give_res")
    return _LinearTM.apply(x, bias, residual, float(dropout_p), in_scale, out_scale, link, *ws)


def ff_tm(x, w1, b1, w2, b2, residual=None, dropout_p: float = 0.0):
    return _FeedForwardTM.apply(x, w1, b1, w2, b2, residual, float(dropout_p))


class _AttentionTM(torch.autograd.Function):
    """Multi-head attention over a fused token-major QKV buffer [B, T, 3C] -> o [B, T, C]."""

    @staticmethod
    def _args(qkv, bias, o, lse, heads, dropout_p=0.0, seed=None):
        B, T, C3 = qkv.shape
        C = C3 // 3
        a = AttnArgs()
        base, es = qkv.data_ptr(), qkv.element_size()
        a.q, a.k, a.v, a.ldq = base, base + C * es, base + 2 * C * es, C3
        a.key_bias, a.o, a.ldo, a.lse = N.ptr(bias), o.data_ptr(), C, lse.data_ptr()
        a.B, a.T, a.H, a.D = B, T, heads, C // heads
        a.scale = 1.0 / math.sqrt(C // heads)
        a.dropout_p, a.seed = float(dropout_p), N.ptr(seed)
        if qkv.dtype == torch.bfloat16:  # bf16 q|k|v (and o, dO, dq|dk|dv): MTTS_ATTN_F_IO_BF16
            if o.dtype != torch.bfloat16:
                raise ValueError("attention: bf16 q|k|v needs a bf16 output")
            a.flags = ATTN_F_IO_BF16
        return a

    @staticmethod
    def forward(ctx, qkv, key_bias, heads, dropout_p):
        _check(qkv, key_bias)
        prec = gemm_precision()
        qkv = _f32c(qkv)
        bias = _f32c(key_bias)
        B, T, C3 = qkv.shape
        o = torch.empty(B, T, C3 // 3, device=qkv.device, dtype=torch.float32)
        lse = torch.empty(B, heads, T, device=qkv.device, dtype=torch.float32)
        seed = _new_seed(qkv.device) if dropout_p > 0 else None
        # precise_forward: exact-fp32 MFMA forward (fp32 q|k|v here), the backward in the region's bf16
        _attn_fwd(qkv, bias, o, lse, heads, PREC_FP32 if _PRECISE.get() else prec, dropout_p, seed)
        ctx.save_for_backward(qkv, bias, o, lse)
        ctx.heads, ctx.prec, ctx.drop = heads, prec, (dropout_p, seed)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, bias, o, lse = ctx.saved_tensors
        return _attn_bwd(_f32c(do), qkv, bias, o, lse, ctx.heads, ctx.prec, *ctx.drop), None, None, None


def _attn_fwd(qkv, bias, o, lse, heads, prec, dropout_p=0.0, seed=None):
    B, T, C3 = qkv.shape
    a = _AttentionTM._args(qkv, bias, o, lse, heads, dropout_p, seed)
    log = ATTN_LOG
    if log is not None:
        st, e0, e1 = _events(qkv.device)
    N.check(N.lib().mtts_attention_fwd(ctypes.byref(a), prec, _stream(qkv)), "mtts_attention_fwd")
    if log is not None:
        e1.record(st)
        D = C3 // 3 // heads
        # two T x T x D products per head; q, k, v read, o and the row statistic written
        log.append((e0, e1, 4.0 * B * heads * T * T * D, prec, 4 * B * T * C3 // 3 * 4 + B * heads * T * 4, "fwd"))


def _attn_bwd(do, qkv, bias, o, lse, heads, prec, dropout_p=0.0, seed=None):
    """-> d(q|k|v) [B, T, 3C] from dO [B, T, C] (in qkv's storage)."""
    B, T, C3 = qkv.shape
    C = C3 // 3
    if do.dtype != qkv.dtype:
        raise ValueError("attention backward: dO must be stored like q|k|v")
    dqkv = torch.empty_like(qkv)
    a = _AttentionTM._args(qkv, bias, o, lse, heads, dropout_p, seed)
    g = AttnGrads()
    g.dout, g.lddo = do.data_ptr(), C
    base, es = dqkv.data_ptr(), dqkv.element_size()
    g.dq, g.dk, g.dv, g.ldd = base, base + C * es, base + 2 * C * es, C3
    lib = N.lib()
    ws = torch.empty(int(lib.mtts_attention_bwd_workspace_size(B, T, heads)), dtype=torch.uint8, device=qkv.device)
    log = ATTN_LOG
    if log is not None:
        st, e0, e1 = _events(qkv.device)
    N.check(lib.mtts_attention_bwd(ctypes.byref(a), ctypes.byref(g), prec, ws.data_ptr(), ws.numel(),
                                   _stream(qkv)), "mtts_attention_bwd")
    if log is not None:
        e1.record(st)
        D = C // heads
        # four T x T x D products per head (dV, dP, dQ, dK; the recomputed S not counted); q, k, v, o,
        # dO, the row statistic read, dq, dk, dv written
        log.append((e0, e1, 8.0 * B * heads * T * T * D, prec, 8 * B * T * C * 4 + B * heads * T * 4, "bwd"))
    return dqkv


def attention_tm(qkv, key_bias, heads: int, dropout_p: float = 0.0):
    """softmax(q k^T / sqrt(d) + key_bias[b, key]) v per head, from the fused projection qkv [B,T,3C]
    (q | k | v column blocks, head h at [h*d, h*d+d) of each); key_bias [B,T].  The reference's float
    0/1 mask is ADDED to the scores (diffusers AttnProcessor2_0 + prepare_attention_mask),
    so padded keys are down-weighted, not removed.  Returns o [B, T, C] token-major."""
    return _AttentionTM.apply(qkv, key_bias, heads, float(dropout_p))


# ------------------------------------------------------------------------------------------ pre-LN sub-blocks
# BasicTransformerBlock (transformer.py:297-370) is two pre-LN residual sub-blocks:
#     h + Dropout(to_out(SDPA(LN1(h) Wq, LN1(h) Wk, LN1(h) Wv)))      and      h + FF(LN3(h)).
# Each runs as ONE autograd Function, so tensors only a GEMM reads can be stored as bf16 in bf16-mixed
# mode (as autocast would hold them) without autograd casting gradients to their dtype: the attention
# block's LayerNorm output (the q|k|v projection's A operand) and the FFN's d(pre-activation) (the dgrad
# GEMM's A, the weight gradient's dY).  The backward adds the residual branch's gradient inside the
# LayerNorm backward (mtts_layernorm_bwd_res) instead of an autograd accumulate kernel per sub-block.
N.register("mtts_layernorm_bwd_res", ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _SZ, _P])
NORM_F_Y_BF16 = 0x100  # include/mtts_decoder.h MTTS_NORM_F_Y_BF16
_PRELN_N16 = os.environ.get("MTTS_PRELN_N16", "1") != "0"  # attention block's LN output as bf16 (A/B switch)
_ATTN_IO16 = os.environ.get("MTTS_ATTN_IO16", "1") != "0"  # bf16 q|k|v / o / dO / dq|dk|dv (A/B switch)
# the FeedForward block's LN output as bf16 (round 5; same-box step A/B 7.546 / 7.531 -> 7.465 / 7.456 ms, bitwise
# the same losses, profiles/r05/ab_preln_ff_n16.txt): the up-projection (now the weight-stationary
# kernel, which rounds an fp32 A to bf16 at the fragment read anyway) and dW1 read it
_PRELN_FF_N16 = os.environ.get("MTTS_PRELN_FF_N16", "1") != "0"


def _ln_fwd(h2, w, b, eps, y16):
    M, C = h2.shape
    n = torch.empty(M, C, device=h2.device, dtype=torch.bfloat16 if y16 else torch.float32)
    mean = torch.empty(M, device=h2.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    N.check(N.lib().mtts_layernorm_fwd(h2.data_ptr(), w.data_ptr(), b.data_ptr(), n.data_ptr(), mean.data_ptr(),
                                       rstd.data_ptr(), M, C, float(eps),
                                       ACT_NONE | (NORM_F_Y_BF16 if n.dtype == torch.bfloat16 else 0), 0.0, None,
                                       _stream(h2)), "mtts_layernorm_fwd")
    return n, mean, rstd


def _ln_bwd_res(dn, h2, w, b, mean, rstd, dres, keys=(None, None)):
    M, C = h2.shape
    dh = torch.empty_like(h2)
    dw = _grad_buf(keys[0], (C,), h2.device)
    db = _grad_buf(keys[1], (C,), h2.device)
    lib = N.lib()
    ws = torch.empty(max(int(lib.mtts_layernorm_bwd_workspace_size(M, C)), 1), dtype=torch.uint8, device=h2.device)
    _keep_partials(ws)
    N.check(lib.mtts_layernorm_bwd_res(dn.data_ptr(), h2.data_ptr(), w.data_ptr(), b.data_ptr(), mean.data_ptr(),
                                       rstd.data_ptr(), dres.data_ptr(), dh.data_ptr(), dw.data_ptr(), db.data_ptr(),
                                       M, C, ws.data_ptr(), ws.numel(), _stream(h2)), "mtts_layernorm_bwd_res")
    return dh, dw, db


class _PreLNAttentionTM(torch.autograd.Function):
    """h + Dropout(to_out(attention(LN1(h) W_qkv))) -- diffusers Attention (AttnProcessor2_0) behind
    BasicTransformerBlock.norm1 (transformer.py:316-331); the float key mask is an additive bias."""

    @staticmethod
    def forward(ctx, h, ln_w, ln_b, eps, key_bias, heads, dropout_p, w_out, b_out, wq, wk, wv):
        _check(h, ln_w, key_bias, w_out, wq)
        prec = gemm_precision()
        shp = h.shape
        h2 = _f32c(h).reshape(-1, shp[-1])
        M, C = h2.shape
        B, T = shp[0], shp[1]
        lnw, lnb = _f32c(ln_w), _f32c(ln_b)
        # (not under precise_forward: its bf16x3 / fp32 GEMMs read the fp32 A's low bits -- ADVICE r5)
        n, mean, rstd = _ln_fwd(h2, lnw, lnb, eps, prec == PREC_BF16 and _PRELN_N16 and not _PRECISE.get())
        Wqkv, Kq = packed(spec_linear((wq, wk, wv)), prec)
        Wo, Ko = packed(spec_linear((w_out,)), prec)
        ctx.wqkv_t = packed(spec_linear((wq, wk, wv), dgrad=True), prec)
        ctx.wo_t = packed(spec_linear((w_out,), dgrad=True), prec)
        C3 = 3 * wq.shape[0]
        # bf16-mixed: q|k|v and o are only MFMA operands (attention, to_out) -- stored bf16
        io16 = prec == PREC_BF16 and _ATTN_IO16 and _bf16_operand_ok(C3 // 3)
        adt = torch.bfloat16 if io16 else torch.float32
        qkv = torch.empty(B, T, C3, device=h.device, dtype=adt)
        _gemm(n, M, M, 1, 1, [0], C, Wqkv, Kq, C3, qkv.view(M, C3), M, prec=prec)
        bias = _f32c(key_bias)
        o = torch.empty(B, T, C3 // 3, device=h.device, dtype=adt)
        lse = torch.empty(B, heads, T, device=h.device, dtype=torch.float32)
        _attn_fwd(qkv, bias, o, lse, heads, prec)
        y = torch.empty(M, C, device=h.device, dtype=torch.float32)
        seed = _new_seed(h.device) if dropout_p > 0 else None
        _gemm(o.view(M, C3 // 3), M, M, 1, 1, [0], C3 // 3, Wo, Ko, C, y, M, prec=prec, bias=_f32c(b_out),
              residual=h2, dropout_p=dropout_p, seed=seed)
        ctx.save_for_backward(h2, lnw, lnb, mean, rstd, n, qkv, bias, o, lse)
        ctx.leaf = _leaves(ln_w, ln_b, w_out, b_out, wq, wk, wv)
        ctx.keys = (_pkey(ln_w), _pkey(ln_b), _pkey(w_out), _pkey(b_out), [_pkey(w) for w in (wq, wk, wv)])
        ctx.cfg = (prec, shp, heads, float(dropout_p), seed, [w.shape for w in (wq, wk, wv)], b_out is not None)
        return y.reshape(shp)

    @staticmethod
    @_grad_sums
    def backward(ctx, dy):
        h2, lnw, lnb, mean, rstd, n, qkv, bias, o, lse = ctx.saved_tensors
        prec, shp, heads, p, seed, qshapes, has_bout = ctx.cfg
        M, C = h2.shape
        B, T, C3 = qkv.shape
        Ci = C3 // 3
        dev = h2.device
        dres = _f32c(dy).reshape(M, C)  # the residual branch's gradient
        g = dres
        if p > 0:  # through to_out's dropout: regenerate the forward's mask
            g = torch.empty_like(dres)
            N.check(N.lib().mtts_dropout_apply(dres.data_ptr(), g.data_ptr(), M, C, C, float(p), seed.data_ptr(),
                                               _stream(g)), "mtts_dropout_apply")
        # to_out: weight + bias gradient, dgrad -> dO
        klw, klb, kwo, kbo, kqkv = ctx.keys
        dwo = _grad_buf(kwo, (C, Ci), dev)
        dbo = _grad_buf(kbo, (C,), dev) if has_bout else None
        _wgrad(g, M, 1, 0, o.view(M, Ci), M, M, 1, 1, [0], Ci, C, dwo, (Ci, 1, 0), prec=prec, db=dbo)
        Wot, Kot = ctx.wo_t
        do = torch.empty(B, T, Ci, device=dev, dtype=qkv.dtype)  # stored like q|k|v
        _gemm(g, M, M, 1, 1, [0], C, Wot, Kot, Ci, do.view(M, Ci), M, prec=prec)
        # attention backward -> d(q|k|v)
        dqkv = _attn_bwd(do, qkv, bias, o, lse, heads, prec)
        # stacked q|k|v projection: weight gradients (A = the bf16 / fp32 LayerNorm output), dgrad -> dn
        dq2 = dqkv.view(M, C3)
        dwqkv = _grad_buf_stacked(kqkv, qshapes, [s_[0] for s_ in qshapes], C, dev)
        _wgrad(dq2, M, 1, 0, n, M, M, 1, 1, [0], C, C3, dwqkv, (C, 1, 0), prec=prec)
        Wqt, Kqt = ctx.wqkv_t
        dn = torch.empty(M, C, device=dev, dtype=torch.float32)
        _gemm(dq2, M, M, 1, 1, [0], C3, Wqt, Kqt, C, dn, M, prec=prec)
        dh, dlnw, dlnb = _ln_bwd_res(dn, h2, lnw, lnb, mean, rstd, dres, (klw, klb))
        dwq, dwk, dwv = (d.view(s_) for d, s_ in zip(dwqkv.split([s_[0] for s_ in qshapes], dim=0), qshapes))
        return dh.reshape(shp), dlnw, dlnb, None, None, None, None, dwo, dbo, dwq, dwk, dwv


class _PreLNFeedForwardTM(torch.autograd.Function):
    """h + Linear2(Dropout(GELU(Linear1(LN3(h))))) -- BasicTransformerBlock.norm3 + FeedForward
    (transformer.py:345-358, :105-188); GELU / dropout / residual in the GEMM epilogues, GELU' folded
    into the second GEMM's dgrad epilogue."""

    @staticmethod
    def forward(ctx, h, ln_w, ln_b, eps, w1, b1, w2, b2, dropout_p):
        _check(h, ln_w, w1, w2)
        prec = gemm_precision()
        shp = h.shape
        h2 = _f32c(h).reshape(-1, shp[-1])
        M, C = h2.shape
        H = w1.shape[0]
        lnw, lnb = _f32c(ln_w), _f32c(ln_b)
        # bf16 LayerNorm output (round 5, _PRELN_FF_N16): the GELU up-projection runs on the weight-stationary
        # kernel, which rounds an fp32 A to bf16 at its fragment read anyway -- the same products, half the bytes
        # (rounds 2-4 kept it fp32: the register-staged schedule then hid the GELU epilogue better)
        # (not under precise_forward, whose split-A GEMMs need the fp32 LN output -- ADVICE r5)
        n, mean, rstd = _ln_fwd(h2, lnw, lnb, eps, prec == PREC_BF16 and _PRELN_FF_N16 and not _PRECISE.get())
        W1p, K1p = packed(spec_linear((w1,), one_plane=not _FF1_SPLIT), prec)
        W2p, K2p = packed(spec_linear((w2,), one_plane=not _FF2_SPLIT), prec)
        ctx.w2t = packed(spec_linear((w2,), dgrad=True), prec)
        ctx.w1t = packed(spec_linear((w1,), dgrad=True), prec)
        b16 = prec == PREC_BF16
        z = torch.empty(M, H, device=h.device, dtype=torch.bfloat16 if b16 else torch.float32)  # pre-activation
        hid = torch.empty(M, H, device=h.device, dtype=torch.bfloat16 if b16 else torch.float32)
        seed = _new_seed(h.device) if dropout_p > 0 else None
        _gemm(n, M, M, 1, 1, [0], C, W1p, K1p, H, hid, M, prec=prec, bias=_f32c(b1), act=ACT_GELU, C_pre=z,
              dropout_p=dropout_p, seed=seed)
        y = torch.empty(M, C, device=h.device, dtype=torch.float32)
        _gemm(hid, M, M, 1, 1, [0], H, W2p, K2p, C, y, M, prec=prec, bias=_f32c(b2), residual=h2)
        ctx.save_for_backward(h2, lnw, lnb, mean, rstd, n, z, hid)
        ctx.leaf = _leaves(ln_w, ln_b, w1, b1, w2, b2)
        ctx.keys = tuple(_pkey(t) for t in (ln_w, ln_b, w1, b1, w2, b2))
        ctx.cfg = (prec, shp, float(dropout_p), seed, w1.shape, w2.shape, b1 is not None, b2 is not None)
        return y.reshape(shp)

    @staticmethod
    @_grad_sums
    def backward(ctx, dy):
        h2, lnw, lnb, mean, rstd, n, z, hid = ctx.saved_tensors
        prec, shp, p, seed, w1s, w2s, has_b1, has_b2 = ctx.cfg
        M, C = h2.shape
        H = w1s[0]
        dev = h2.device
        dy2 = _f32c(dy).reshape(M, C)  # also the residual branch's gradient
        klw, klb, kw1, kb1, kw2, kb2 = ctx.keys
        dw2 = _grad_buf(kw2, w2s, dev)
        db2 = _grad_buf(kb2, (C,), dev) if has_b2 else None
        _wgrad(dy2, M, 1, 0, hid, M, M, 1, 1, [0], H, C, dw2, (H, 1, 0), prec=prec, db=db2)
        W2t, K2p = ctx.w2t
        # d(pre-activation): bf16 in bf16-mixed -- only the next dgrad GEMM and dW1 read it
        dz = torch.empty(M, H, device=dev, dtype=torch.bfloat16 if prec == PREC_BF16 else torch.float32)
        _gemm(dy2, M, M, 1, 1, [0], C, W2t, K2p, H, dz, M, prec=prec, act=ACT_DGELU, aux=z, dropout_p=p, seed=seed)
        dw1 = _grad_buf(kw1, w1s, dev)
        db1 = _grad_buf(kb1, (H,), dev) if has_b1 else None
        _wgrad(dz, M, 1, 0, n, M, M, 1, 1, [0], C, H, dw1, (C, 1, 0), prec=prec, db=db1)
        W1t, K1p = ctx.w1t
        dn = torch.empty(M, C, device=dev, dtype=torch.float32)
        _gemm(dz, M, M, 1, 1, [0], H, W1t, K1p, C, dn, M, prec=prec)
        dh, dlnw, dlnb = _ln_bwd_res(dn, h2, lnw, lnb, mean, rstd, dy2, (klw, klb))
        return dh.reshape(shp), dlnw, dlnb, None, dw1, db1, dw2, db2, None


def preln_attention_tm(h, ln_w, ln_b, eps, key_bias, heads, wq, wk, wv, w_out, b_out, dropout_p: float = 0.0):
    """h + Dropout(to_out(SDPA(q, k, v, key bias))), q|k|v = LN(h) [Wq; Wk; Wv]^T (no bias), token-major."""
    return _PreLNAttentionTM.apply(h, ln_w, ln_b, float(eps), key_bias, int(heads), float(dropout_p), w_out, b_out,
                                   wq, wk, wv)


def preln_ff_tm(h, ln_w, ln_b, eps, w1, b1, w2, b2, dropout_p: float = 0.0):
    """h + W2 Dropout(GELU(W1 LN(h) + b1)) + b2, token-major."""
    return _PreLNFeedForwardTM.apply(h, ln_w, ln_b, float(eps), w1, b1, w2, b2, float(dropout_p))


class _RopeTM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, heads, rope_dims):
        _check(qkv, cos, sin)
        qkv, cos, sin = _f32c(qkv), _f32c(cos), _f32c(sin)  # the kernel reads fp32 tables [T, rope_dims/2]
        assert cos.shape == sin.shape == (qkv.shape[1], rope_dims // 2)
        B, T, C3 = qkv.shape
        out = torch.empty_like(qkv)
        N.check(N.lib().mtts_rope_qk(qkv.data_ptr(), out.data_ptr(), B * T, T, C3 // 3, heads, rope_dims,
                                     cos.data_ptr(), sin.data_ptr(), 0, _stream(qkv)), "mtts_rope_qk")
        ctx.save_for_backward(cos, sin)
        ctx.cfg = (heads, rope_dims)
        return out

    @staticmethod
    def backward(ctx, dout):
        cos, sin = ctx.saved_tensors
        heads, rope_dims = ctx.cfg
        dout = _f32c(dout)
        B, T, C3 = dout.shape
        dx = torch.empty_like(dout)
        N.check(N.lib().mtts_rope_qk(dout.data_ptr(), dx.data_ptr(), B * T, T, C3 // 3, heads, rope_dims,
                                     cos.data_ptr(), sin.data_ptr(), 1, _stream(dout)), "mtts_rope_qk")
        return dx, None, None, None, None


def rope_tm(qkv, cos, sin, heads: int, rope_dims: int):
    """Rotary embedding of the q and k blocks of a fused [B, T, 3C] projection (first rope_dims dims of
    each head, rotate-half form; cos/sin [T, rope_dims/2]); v passes through."""
    return _RopeTM.apply(qkv, cos, sin, heads, rope_dims)


# ------------------------------------------------------------------------------------------ step glue
N.register("mtts_sequence_mask_f32", ctypes.c_int, [_P, _I, _I, _P, _P, _P])
N.register("mtts_duration_loss_fwd", ctypes.c_int, [_P, _P, _P, _I, _I, _P, _P])
N.register("mtts_duration_loss_bwd", ctypes.c_int, [_P, _P, _P, _P, _P, _I, _I, _P, _P])
N.register("mtts_loss_sum", ctypes.c_int, [_P, _P, _P, _P, _P, _P])


def _lengths64(lengths: torch.Tensor) -> torch.Tensor:
    return lengths if (lengths.dtype == torch.int64 and lengths.is_contiguous()) else lengths.to(torch.int64).contiguous()


def sequence_mask_f32(lengths: torch.Tensor, T: int, key_bias: bool = False):
    """fp32 0/1 mask [B, T] of utils/model.py:13-34 sequence_mask(lengths, T).float() in one launch; with
    key_bias=True also (mask - 1) * 1e4 (the text encoder's masked_fill(-1e4) as an additive key bias):
    returns (mask, bias)."""
    N.require_device(lengths)
    ln = _lengths64(lengths)
    B = ln.numel()
    m = torch.empty(B, T, dtype=torch.float32, device=ln.device)
    kb = torch.empty(B, T, dtype=torch.float32, device=ln.device) if key_bias else None
    N.check(N.lib().mtts_sequence_mask_f32(ln.data_ptr(), B, T, m.data_ptr(), N.ptr(kb), _stream(ln)),
            "mtts_sequence_mask_f32")
    return (m, kb) if key_bias else m


class _DurationLoss(torch.autograd.Function):
    """sum((logw - log(1e-8 + dur) * x_mask)^2) / sum(x_lengths) -- matcha_tts.py:287-288 + utils/model.py:117-135
    in one launch forward and one backward (csrc/losses.hip); dur (the MAS durations) has no gradient."""

    @staticmethod
    def forward(ctx, logw, dur, lengths):
        N.require_device(logw, dur, lengths)
        B, T = dur.shape[0], dur.shape[-1]
        lw, d, ln = _f32c(logw).reshape(B, T), _f32c(dur).reshape(B, T), _lengths64(lengths)
        out = torch.empty(2, dtype=torch.float32, device=lw.device)
        N.check(N.lib().mtts_duration_loss_fwd(lw.data_ptr(), d.data_ptr(), ln.data_ptr(), B, T, out.data_ptr(),
                                               _stream(lw)), "mtts_duration_loss_fwd")
        ctx.save_for_backward(lw, d, ln, out)
        ctx.shape = logw.shape
        return out[0]

    @staticmethod
    def backward(ctx, g):
        lw, d, ln, out = ctx.saved_tensors
        B, T = d.shape
        g = _f32c(g)
        dlogw = torch.empty_like(lw)
        N.check(N.lib().mtts_duration_loss_bwd(g.data_ptr(), out.data_ptr(), lw.data_ptr(), d.data_ptr(), ln.data_ptr(),
                                               B, T, dlogw.data_ptr(), _stream(lw)), "mtts_duration_loss_bwd")
        return dlogw.view(ctx.shape), None, None


def duration_loss_fused(logw: torch.Tensor, dur: torch.Tensor, lengths: torch.Tensor) -> torch.Tensor:
    """logw [B, 1, T] (the duration predictor's output), dur [B, T] -> the duration loss (0-dim fp32)."""
    return _DurationLoss.apply(logw, dur, lengths)


class _LossSum(torch.autograd.Function):
    """total = (dur + prior) + diff and the logged vector [dur, prior, diff, total] in one launch
    (baselightningmodule.py:121-128); the gradient of total reaches each loss unchanged."""

    @staticmethod
    def forward(ctx, dur, prior, diff):
        N.require_device(dur, diff)
        dur, diff = _f32c(dur), _f32c(diff)
        prior = _f32c(prior) if torch.is_tensor(prior) else None
        total = torch.empty((), dtype=torch.float32, device=dur.device)
        logged = torch.empty(4, dtype=torch.float32, device=dur.device)
        N.check(N.lib().mtts_loss_sum(dur.data_ptr(), N.ptr(prior), diff.data_ptr(), total.data_ptr(), logged.data_ptr(),
                                      _stream(dur)), "mtts_loss_sum")
        ctx.has_prior = prior is not None
        ctx.mark_non_differentiable(logged)
        return total, logged

    @staticmethod
    def backward(ctx, g, _g_logged):
        return g, (g if ctx.has_prior else None), g


def loss_sum(dur, prior, diff):
    """(total, logged): total = dur + prior + diff (prior may be the int 0 of prior_loss=False)."""
    return _LossSum.apply(dur, prior if torch.is_tensor(prior) else None, diff)


# ------------------------------------------------------------------------------------------ time MLP
N.register("mtts_rows_linear_workspace_size", _SZ, [_I, _I, _I, _P])
N.register("mtts_rows_linear_fwd", ctypes.c_int, [_P, _I, _I, _I, _P, _P, _P, _P, _P, _I, _P, _SZ, _P])
N.register("mtts_rows_linear_bwd", ctypes.c_int, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _SZ, _P])
ROWS_ACT_NONE, ROWS_ACT_SILU, ROWS_ACT_MISH = 0, 1, 2  # include/mtts_decoder.h MTTS_ROWS_ACT_*


def _ptrs(ts):
    return (ctypes.c_void_p * len(ts))(*[None if t is None else t.data_ptr() for t in ts])


# per (device, B, K, N...) workspaces of the rows GEMMs: the counter region is zeroed once here and left
# zeroed by the kernels, so a captured graph replays with the same buffers (never freed: a few hundred KB)
_ROWS_WS: dict = {}


def _rows_ws(dev, B, K, ns):
    key = (dev, B, K, tuple(ns))
    t = _ROWS_WS.get(key)
    if t is None:
        arr = (ctypes.c_int32 * len(ns))(*ns)
        nb = int(N.lib().mtts_rows_linear_workspace_size(B, K, len(ns), arr))
        t = torch.zeros(max(nb, 256) // 4 + 64, dtype=torch.float32, device=dev)
        _ROWS_WS[key] = t
    return t


ROWS_MAX_MATS = 8  # include/mtts_decoder.h MTTS_ROWS_MAX_MATS: matrices per rows-linear launch


def _chunks(n):
    return [(i, min(i + ROWS_MAX_MATS, n)) for i in range(0, n, ROWS_MAX_MATS)]


def _rows_fwd(x, ws, bs, outs, acts, act):
    """out_i = x W_i^T + b_i (act_i = act(out_i)); more than ROWS_MAX_MATS matrices run as several launches."""
    if len(ws) > ROWS_MAX_MATS:
        for i, j in _chunks(len(ws)):
            _rows_fwd(x, ws[i:j], bs[i:j], outs[i:j], None if acts is None else acts[i:j], act)
        return
    B, K = x.shape
    nl = [w.shape[0] for w in ws]
    wsb = _rows_ws(x.device, B, K, nl)
    ns = (ctypes.c_int32 * len(ws))(*nl)
    N.check(N.lib().mtts_rows_linear_fwd(x.data_ptr(), B, K, len(ws), _ptrs(ws), _ptrs(bs), ns, _ptrs(outs),
                                         None if acts is None else _ptrs(acts), act, wsb.data_ptr(),
                                         wsb.numel() * 4, _stream(x)), "mtts_rows_linear_fwd")


def _rows_bwd(a, pre, act, ws, dys, dx, dws, dbs):
    """Backward of _rows_fwd.  More than ROWS_MAX_MATS matrices: one launch per chunk, and the chunks'
    input gradients (each already times act'(pre)) summed in chunk order."""
    if len(ws) > ROWS_MAX_MATS:
        part = None if dx is None else torch.empty_like(dx)
        for c, (i, j) in enumerate(_chunks(len(ws))):
            _rows_bwd(a, pre, act, ws[i:j], dys[i:j], dx if c == 0 else part, dws[i:j], dbs[i:j])
            if c > 0 and dx is not None:
                dx.add_(part)
        return
    B, K = a.shape
    nl = [w.shape[0] for w in ws]
    wsb = _rows_ws(a.device, B, K, nl)
    ns = (ctypes.c_int32 * len(ws))(*nl)
    N.check(N.lib().mtts_rows_linear_bwd(a.data_ptr(), N.ptr(pre), act, B, K, len(ws), _ptrs(ws), ns, _ptrs(dys),
                                         N.ptr(dx), _ptrs(dws), _ptrs(dbs), wsb.data_ptr(), wsb.numel() * 4,
                                         _stream(a)), "mtts_rows_linear_bwd")


class _TimeMLP(torch.autograd.Function):
    """e [B, in] -> (temb, tp_0 .. tp_{n-1}): TimeStepEmbeddingNet (decoder.py:33-49, Linear -> SiLU ->
    Linear) and every Resnet1D.mlp (decoder.py:71-72, 80-81, Mish -> Linear) on the shared temb, in fp32,
    3 launches forward and 5 backward (csrc/time_mlp.hip).  The projections are one matrix table: no
    weight concatenation, each tp_i is written contiguous."""

    @staticmethod
    def forward(ctx, e, w1, b1, w2, b2, n_proj, pre, *wb):
        N.require_device(e, w1)
        ctx.keys = ([_pkey(t) for t in (w1, b1, w2, b2)], [_pkey(w) for w in wb[:n_proj]],
                    [_pkey(b) for b in wb[n_proj:]])
        ws = [_f32c(w) for w in wb[:n_proj]]
        bs = [_f32c(b) for b in wb[n_proj:]]
        e, w1, b1, w2, b2 = _f32c(e), _f32c(w1), _f32c(b1), _f32c(w2), _f32c(b2)
        if pre is not None:  # launched ahead on the side stream (time_mlp_launch); the caller has joined it
            h1, a1, temb, a2, tps = pre
        else:
            h1, a1, temb, a2, tps = _time_mlp_launch(e, w1, b1, w2, b2, ws, bs, _time_mlp_alloc(e, w1, b1, w2, b2, ws, bs))
        ctx.save_for_backward(e, h1, a1, temb, a2, w1, w2, *ws)
        ctx.n = n_proj
        ctx.e_grad = ctx.needs_input_grad[0]
        ctx.set_materialize_grads(False)
        return (temb, *tps)

    @staticmethod
    def backward(ctx, g_temb, *g_tps):
        e, h1, a1, temb, a2, w1, w2, *ws = ctx.saved_tensors
        B, D = temb.shape
        new = functools.partial(torch.empty, dtype=torch.float32, device=e.device)
        dys = [_f32c(g) if g is not None else torch.zeros(B, w.shape[0], device=e.device) for g, w in zip(g_tps, ws)]
        d_temb = new(B, D)
        (k1, kb1, k2, kb2), kws, kbs = ctx.keys  # data-parallel grad slots (else fresh buffers)
        dws = [_grad_buf(k, w.shape, e.device) for k, w in zip(kws, ws)]
        dbs = [_grad_buf(k, (w.shape[0],), e.device) for k, w in zip(kbs, ws)]
        dh1, dw2, db2 = new(B, D), _grad_buf(k2, w2.shape, e.device), _grad_buf(kb2, (D,), e.device)
        de = new(*e.shape) if ctx.e_grad else None
        dw1, db1 = _grad_buf(k1, w1.shape, e.device), _grad_buf(kb1, (D,), e.device)
        # on the decoder's path (t carries no gradient) every output is a parameter gradient: the five
        # launches leave the critical path for the deferral's side stream (joined before the optimizer)
        # -- only when autograd takes EVERY output as a parameter gradient: it then steals each tensor (no
        # kernel) and nothing reads it before the join.  The outputs are NOT kept alive here: an extra
        # reference makes AccumulateGrad copy the gradient on the main stream while the side kernels still
        # write it (zeros in a replayed graph, tests/test_training_gpu.py::
        # test_graph_gradients_equal_eager_over_replays); a frozen weight (needs_input_grad False) would have
        # its gradient dropped at once and its memory reused under the side kernels, so that case stays on
        # the main stream
        all_params = all(ctx.needs_input_grad[1:5]) and all(ctx.needs_input_grad[7:])
        side = param_grad_side_stream() if (not ctx.e_grad and g_temb is None and all_params) else None
        if side is not None:
            keep_for_side(e, h1, a1, temb, a2, w1, w2, *ws, *dys, d_temb, dh1)
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            _rows_bwd(a2, temb, ROWS_ACT_MISH, ws, dys, d_temb, dws, dbs)
            if g_temb is not None:  # temb used directly as well (never, on the decoder's path)
                d_temb = d_temb + _f32c(g_temb)
            _rows_bwd(a1, h1, ROWS_ACT_SILU, [w2], [d_temb], dh1, [dw2], [db2])
            _rows_bwd(e, None, ROWS_ACT_NONE, [w1], [dh1], de, [dw1], [db1])
        return (de, dw1, db1, dw2, db2, None, None, *dws, *dbs)


def _time_mlp_alloc(e, w1, b1, w2, b2, ws, bs):
    """The forward's outputs, allocated on the current stream (a caller may then launch under another)."""
    B, D = e.shape[0], w1.shape[0]
    new = functools.partial(torch.empty, dtype=torch.float32, device=e.device)
    h1, a1, temb, a2 = new(B, D), new(B, D), new(B, D), new(B, D)
    tps = [new(B, w.shape[0]) for w in ws]
    return h1, a1, temb, a2, tps


def _time_mlp_launch(e, w1, b1, w2, b2, ws, bs, outs):
    h1, a1, temb, a2, tps = outs
    _rows_fwd(e, [w1], [b1], [h1], [a1], ROWS_ACT_SILU)
    _rows_fwd(a1, [w2], [b2], [temb], [a2], ROWS_ACT_MISH)
    _rows_fwd(a2, ws, bs, tps, None, ROWS_ACT_NONE)
    return outs


def time_mlp(e, linear_1, linear_2, proj_linears, pre=None):
    """(temb, [tp_i]) = (time_mlp(e), [lin_i(mish(temb))]) for nn.Linear modules; see _TimeMLP.  pre: the
    forward's tensors from time_mlp_ahead (already joined)."""
    ws = [lin.weight for lin in proj_linears]
    bs = [lin.bias for lin in proj_linears]
    out = _TimeMLP.apply(e, linear_1.weight, linear_1.bias, linear_2.weight, linear_2.bias, len(ws), pre, *ws, *bs)
    return out[0], list(out[1:])


def time_mlp_ahead(e, linear_1, linear_2, proj_linears, side):
    """The time MLP's forward launched on `side` now (outputs allocated on the current stream) -> the
    `pre` tensors for time_mlp once the caller has joined `side`."""
    w1, b1, w2, b2 = (_f32c(v) for v in (linear_1.weight, linear_1.bias, linear_2.weight, linear_2.bias))
    ws = [_f32c(lin.weight) for lin in proj_linears]
    bs = [_f32c(lin.bias) for lin in proj_linears]
    outs = _time_mlp_alloc(e, w1, b1, w2, b2, ws, bs)
    keep_for_side(e, w1, b1, w2, b2, *ws, *bs, *outs[:4], *outs[4])  # alive until the side stream is joined
    with torch.cuda.stream(side):
        _time_mlp_launch(e, w1, b1, w2, b2, ws, bs, outs)
    return outs
