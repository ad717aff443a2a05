// Shared helpers for the libmtts_hip.so translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mtts_base.h"
#include "mtts_decoder.h"

namespace mtts {

// Counter-based dropout keep test shared by the GEMM epilogues, the norms, the attention probabilities
// and mtts_dropout_apply: one murmur3 finalizer over a (row, column pair, seed) key, whose two 16-bit halves
// are the uniforms of the pair's even and odd column.  32-bit integer multiplies run at a quarter of the VALU
// rate on CDNA; the row product is loop-invariant in the epilogues (hoisted) and the 16-byte epilogues hand
// adjacent column pairs to one hash (the compiler merges the identical calls): one finalizer per two elements
// (round 5: the FeedForward GELU epilogue spent ~35 % of its VALU cycles in the per-element hash).  The keep
// probability is quantised to the 2^-16 grid: an element is kept iff u >= ceil(p * 65536), so P(keep) =
// (65536 - ceil(p * 65536)) / 65536 (p = 0.1: 0.899994), and dropout_scale() rescales by exactly its inverse --
// E[kept * scale] = 1 with no grid bias.  Every site that regenerates a mask calls this with the same
// (row, col), so forward and backward agree.
__device__ __forceinline__ bool dropout_keep(uint32_t seed_lo, uint32_t seed_hi, uint32_t row, uint32_t col,
                                             float p) {
    uint32_t x = ((row * 0x9E3779B1u) ^ (((col >> 1) + 0x7F4A7C15u) * 0x85EBCA77u) ^ seed_lo) + seed_hi;
    x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
    const uint32_t u = (col & 1u) ? (x >> 16) : (x & 0xFFFFu);
    return (float)u * (1.0f / 65536.0f) >= p;
}

// 1 / P(keep) of dropout_keep: 65536 / (65536 - ceil(p * 65536)) (p * 65536 is exact in fp32); 1 at p <= 0
__host__ __device__ __forceinline__ float dropout_scale(float p) {
    return p > 0.f ? 65536.0f / (65536.0f - ceilf(p * 65536.0f)) : 1.0f;
}

// Tap offset j of a conv argument struct (static indexing only: no private-memory copy of off[]).
template <class P>
__device__ __forceinline__ int tap_off(const P &p, int j) {
    int o = p.off[0];
#pragma unroll
    for (int i = 1; i < MTTS_CONV_MAX_TAPS; ++i) o = j == i ? p.off[i] : o;
    return o;
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
