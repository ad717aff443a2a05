// conv_gemm_wreg.hip / conv_gemm_wreg16.hip: weight-stationary bf16 schedules of mtts_conv_gemm (ids MTTS_GEMM_WREG, + 1)
#pragma once

#include <hip/hip_runtime.h>

#include "mtts_decoder.h"

namespace mtts {
bool conv_gemm_wreg_applies(const mtts_conv_gemm_args &p);
// the heuristic's choice: every row stream takes >= 2 tiles, or the whole grid is one round of workgroups
bool conv_gemm_wreg_preferred(const mtts_conv_gemm_args &p, int M);
int conv_gemm_wreg_launch(const mtts_conv_gemm_args &p, int M, hipStream_t st);
// conv_gemm_wreg16.hip (id MTTS_GEMM_WREG + 1): 16 columns per wave, K = 768 (k = 3 convs over 256 channels), 512,
// 1024 (linears); bf16 A
bool conv_gemm_wreg16_applies(const mtts_conv_gemm_args &p);
bool conv_gemm_wreg16_preferred(const mtts_conv_gemm_args &p, int M);
int conv_gemm_wreg16_launch(const mtts_conv_gemm_args &p, int M, hipStream_t st);
}  // namespace mtts
