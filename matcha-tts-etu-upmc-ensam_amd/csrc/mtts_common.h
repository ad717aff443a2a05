// Shared helpers for the libmtts_hip.so translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mtts.h"
#include "mtts_decoder.h"

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

// Tap offset j of a conv argument struct (static indexing only: no private-memory copy of off[]).
template <class P>
__device__ __forceinline__ int tap_off(const P &p, int j) {
    int o = p.off[0];
#pragma unroll
    for (int i = 1; i < MTTS_CONV_MAX_TAPS; ++i) o = j == i ? p.off[i] : o;
    return o;
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

// d/dx erf-GELU, as torch's GeluBackward (cdf + x * pdf)
__device__ __forceinline__ float gelu_erf_grad(float x) {
    const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
    const float pdf = expf(-0.5f * x * x) * 0.39894228040143268f;
    return cdf + x * pdf;
}

// erf-GELU / GELU' with erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7; 5.2e-7 evaluated in fp32) sharing ONE exponential
// between erf and the normal pdf: for the bf16-mixed GEMM epilogues (MTTS_GEMM_F_FAST_ACT), where the
// result is rounded to a bf16 operand anyway; erff (torch's erf to an ulp) made the 1024-wide FFN
// epilogues VALU-heavy.  The fp32 parity mode keeps erff.
__device__ __forceinline__ float erf_as_pdf(float z, float &ez2) {  // erf(z), ez2 = exp(-z^2)
    const float a = fabsf(z);
    const float t = __frcp_rn(1.f + 0.3275911f * a);
    ez2 = __expf(-a * a);
    const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
    const float r = 1.f - poly * ez2;
    return copysignf(r, z);
}
__device__ __forceinline__ float gelu_fast(float x) {
    float e;
    return 0.5f * x * (1.0f + erf_as_pdf(x * 0.70710678118654752f, e));
}
__device__ __forceinline__ float gelu_grad_fast(float x) {
    float e;  // exp(-x^2/2)
    const float cdf = 0.5f * (1.0f + erf_as_pdf(x * 0.70710678118654752f, e));
    return cdf + x * e * 0.39894228040143268f;
}

// GEMM epilogue activation (include/mtts_decoder.h MTTS_ACT_*); aux is read only by the D-variants.
__device__ __forceinline__ float epi_act(int act, float v, const float *aux, bool fast = false) {
    switch (act) {
        case MTTS_ACT_GELU: return fast ? gelu_fast(v) : gelu_erf(v);
        case MTTS_ACT_DGELU: return v * (fast ? gelu_grad_fast(*aux) : gelu_erf_grad(*aux));
        case MTTS_ACT_RELU: return fmaxf(v, 0.f);
        case MTTS_ACT_DRELU: return *aux > 0.f ? v : 0.f;
        default: return v;
    }
}

}  // namespace mtts

struct mtts_conv_gemm_args;
namespace mtts {
// conv_gemm_glds.hip: bf16 LDS-DMA schedules (ids MTTS_GEMM_GLDS + 0 .. num - 1)
int conv_gemm_glds_num_cfgs();
bool conv_gemm_glds_applies(const mtts_conv_gemm_args &p);
bool conv_gemm_glds_lean(const mtts_conv_gemm_args &p);  // whole-tap K steps: scalar-addressed loop
// splits > 1: split-K into `part` (conv_gemm_glds_splitk_bytes of workspace) + a combine/epilogue pass
int conv_gemm_glds_launch(int id, const mtts_conv_gemm_args &p, int M, int splits, float *part, hipStream_t st);
size_t conv_gemm_glds_splitk_bytes(const mtts_conv_gemm_args &p, int splits);
}  // namespace mtts

struct mtts_reduce_job;
namespace mtts {
// reduce.hip: runs the partial-sum jobs now, or queues them while deferral is on
int submit_reductions(const mtts_reduce_job *jobs, int njobs, hipStream_t st);
// reduce.hip: appends jobs to the deferred queue whatever the deferral state (the next flush runs them)
int queue_reductions(const mtts_reduce_job *jobs, int njobs);
// reduce.hip: deferral currently on (mtts_defer_reductions)
bool deferring();
// conv_gemm.hip: the deferred weight gradients -- launched batched (their slab sums then queued), counted
// as the slab sums they will add, dropped
int flush_wgrads(hipStream_t st);
int pending_wgrad_sums();
void discard_wgrads();
}  // namespace mtts

#define MTTS_CHECK_ARG(cond, msg)                                   \
    do {                                                            \
        if (!(cond)) return ::mtts::fail(MTTS_ERR_INVALID_ARG, msg); \
    } while (0)
