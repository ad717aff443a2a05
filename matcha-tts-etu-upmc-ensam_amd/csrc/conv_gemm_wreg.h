// conv_gemm_wreg.hip: the weight-stationary bf16 schedule of mtts_conv_gemm (id MTTS_GEMM_WREG, W in registers)
#pragma once

#include <hip/hip_runtime.h>

#include "mtts_decoder.h"

namespace mtts {
bool conv_gemm_wreg_applies(const mtts_conv_gemm_args &p);
// the heuristic's choice: every row stream takes >= 2 tiles, or the whole grid is one round of workgroups
bool conv_gemm_wreg_preferred(const mtts_conv_gemm_args &p, int M);
int conv_gemm_wreg_launch(const mtts_conv_gemm_args &p, int M, hipStream_t st);
}  // namespace mtts
