// Shared helpers for the libmtts_hip.so translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mtts_base.h"
#include "mtts_decoder.h"

namespace mtts {

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
