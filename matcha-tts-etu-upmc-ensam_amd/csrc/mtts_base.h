// Base helpers of the libmtts_hip.so translation units that need only the MAS ABI (include/mtts.h): error slot,
// launch checks, the dropout hash, the LDS-only barrier.  mas.hip includes this alone, so that a change to the
// decoder ABI header (include/mtts_decoder.h) does not rebuild it (its device compile is most of a full build).
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

// Counter-based dropout keep test shared by the GEMM epilogues, the norms, the attention probabilities
// and mtts_dropout_apply: one murmur3 finalizer over a (row, col, seed) key.  32-bit integer multiplies
// run at a quarter of the VALU rate on CDNA; the row and column products are loop-invariant in the
// epilogues (hoisted), leaving two per element instead of the two-round form's four (train step
// 8.97 -> 8.92 ms, tools/gpu_lib_ab.sh).  The keep probability is exactly 1 - p up to the 2^-24 grid.
__device__ __forceinline__ bool dropout_keep(uint32_t seed_lo, uint32_t seed_hi, uint32_t row, uint32_t col,
                                             float p) {
    uint32_t x = ((row * 0x9E3779B1u) ^ ((col + 0x7F4A7C15u) * 0x85EBCA77u) ^ seed_lo) + seed_hi;
    x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
    return (float)(x >> 8) * (1.0f / 16777216.0f) >= p;
}

// Workgroup barrier for an LDS hand-off only: waits for this wave's LDS operations, NOT for its
// outstanding global loads.  __syncthreads() carries a fence that makes hipcc drain vmcnt before the
// s_barrier, which would turn every register prefetch into a synchronous load.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

}  // namespace mtts

#define MTTS_CHECK_ARG(cond, msg)                                   \
    do {                                                            \
        if (!(cond)) return ::mtts::fail(MTTS_ERR_INVALID_ARG, msg); \
    } while (0)
