// Shared helpers for the libmtts_hip.so translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mtts.h"

namespace mtts {

// Records a printf-style message in the calling thread's error slot (read by mtts_last_error).
void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

inline int fail(int code, const char *msg) {
    set_error("%s", msg);
    return code;
}

inline int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return MTTS_ERR_HIP;
    }
    return MTTS_OK;
}

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Counter-based dropout keep test shared by the GEMM epilogue and mtts_dropout_apply.
__device__ __forceinline__ bool dropout_keep(uint32_t seed_lo, uint32_t seed_hi, uint32_t row, uint32_t col,
                                             float p) {
    uint32_t x = row * 0x9E3779B1u ^ (col + 0x7F4A7C15u) * 0x85EBCA77u ^ seed_lo;
    x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
    x ^= seed_hi;
    x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
    return (float)(x >> 8) * (1.0f / 16777216.0f) >= p;
}

}  // namespace mtts

struct mtts_conv_gemm_args;
namespace mtts {
// conv_gemm_panel.hip: A-resident bf16 schedule; returns 0 if launched, 1 if it does not apply.
int conv_gemm_panel_launch(const mtts_conv_gemm_args &p, hipStream_t st);
}  // namespace mtts

#define MTTS_CHECK_ARG(cond, msg)                                   \
    do {                                                            \
        if (!(cond)) return ::mtts::fail(MTTS_ERR_INVALID_ARG, msg); \
    } while (0)
