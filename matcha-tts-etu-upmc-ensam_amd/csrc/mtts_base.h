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
