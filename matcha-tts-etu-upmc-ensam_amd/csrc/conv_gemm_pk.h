// conv_gemm_pk.hip: persistent big-tile LDS-DMA schedules of mtts_conv_gemm (ids MTTS_GEMM_PK + 0 .. num - 1)
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

#include "mtts_decoder.h"

namespace mtts {
int conv_gemm_pk_num_cfgs();
// f32: exact-fp32 operands and MFMA (MTTS_PREC_FP32), else bf16 MFMA on one or two weight planes
bool conv_gemm_pk_applies(int id, const mtts_conv_gemm_args &p, bool f32);
// the tail tiles run stream-K when the workspace holds conv_gemm_pk_workspace_bytes (else every tile whole)
size_t conv_gemm_pk_workspace_bytes(int id, const mtts_conv_gemm_args &p, bool f32);
int conv_gemm_pk_launch(int id, const mtts_conv_gemm_args &p, int M, void *ws, size_t ws_bytes, hipStream_t st, bool f32);
}  // namespace mtts
