// Token embedding of the text encoder (text_encoder.py:341-342, :389):
//   out[r, :] = W[ids[r], :] * scale            (nn.Embedding lookup, then * sqrt(C))
// and its weight gradient
//   dW[v, :] = sum over rows r with ids[r] == v, in ascending r, of (dout[r, :] * scale)
// torch's embedding backward on the GPU sums with atomics (a run-to-run varying order); here one
// workgroup per vocabulary entry walks the rows in index order, so the gradient is deterministic and
// the whole training step bit-reproducible.  Each term is rounded as torch rounds it (the scale
// product first, then the sum): -ffp-contract is irrelevant, the product and sum are separate ops.
//
// Rows are scanned 256 at a time: every thread tests one id, the matches of the chunk are compacted
// into LDS in row order (wave ballots + popcount prefixes), then each thread adds its channels over
// the compacted rows.  ids are read V times from L2 (8 B x rows x V: 4.6 MB at B=32, Tx=120, V=150),
// dout once.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mtts_common.h"

namespace {

constexpr int kEThreads = 256;

__global__ __launch_bounds__(kEThreads) void embedding_fwd_kernel(const int64_t *__restrict__ ids,
                                                                   const float *__restrict__ w, int64_t rows, int C,
                                                                   int V, float scale, float *__restrict__ out) {
    const int64_t r = blockIdx.x;
    if (r >= rows) return;
    int64_t v = ids[r];
    v = v < 0 ? 0 : (v >= V ? V - 1 : v);  // ids are validated on the host; clamp keeps reads in bounds
    const float *src = w + v * C;
    float *dst = out + r * C;
    for (int c = threadIdx.x; c < C; c += blockDim.x) dst[c] = src[c] * scale;
}

__global__ __launch_bounds__(kEThreads) void embedding_bwd_kernel(const int64_t *__restrict__ ids,
                                                                   const float *__restrict__ dout, int64_t rows,
                                                                   int C, float scale, float *__restrict__ dw) {
    __shared__ int s_rows[kEThreads];
    __shared__ int s_wave_cnt[kEThreads / 64];
    const int v = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int kMaxCPerThread = 4;  // C <= 1024 (checked on the host)
    float acc[kMaxCPerThread];
#pragma unroll
    for (int i = 0; i < kMaxCPerThread; ++i) acc[i] = 0.f;
    for (int64_t r0 = 0; r0 < rows; r0 += kEThreads) {
        const int64_t r = r0 + threadIdx.x;
        const bool hit = r < rows && ids[r] == v;
        const uint64_t m = __ballot(hit);
        if (lane == 0) s_wave_cnt[wave] = __popcll(m);
        __syncthreads();
        int base = 0, total = 0;
#pragma unroll
        for (int w = 0; w < kEThreads / 64; ++w) {
            const int c = s_wave_cnt[w];
            base += w < wave ? c : 0;
            total += c;
        }
        if (hit) s_rows[base + __popcll(m & ((1ull << lane) - 1ull))] = (int)(r - r0);
        __syncthreads();
        for (int k = 0; k < total; ++k) {
            const float *src = dout + (r0 + s_rows[k]) * C;
#pragma unroll
            for (int i = 0; i < kMaxCPerThread; ++i) {
                const int c = threadIdx.x + i * kEThreads;
                if (c < C) acc[i] += src[c] * scale;
            }
        }
        __syncthreads();  // s_rows / s_wave_cnt are rewritten by the next chunk
    }
#pragma unroll
    for (int i = 0; i < kMaxCPerThread; ++i) {
        const int c = threadIdx.x + i * kEThreads;
        if (c < C) dw[(int64_t)v * C + c] = acc[i];
    }
}

}  // namespace

extern "C" int mtts_embedding_fwd(const int64_t *ids, const float *weight, int64_t rows, int32_t V, int32_t C,
                                  float scale, float *out, void *hip_stream) {
    MTTS_CHECK_ARG(ids && weight && out && rows >= 0 && V >= 1 && C >= 1 && rows <= 0x7fffffff,
                   "embedding_fwd: bad args");
    if (rows == 0) return MTTS_OK;
    hipLaunchKernelGGL(embedding_fwd_kernel, dim3((unsigned)rows), dim3(C >= 256 ? 256 : 64 * ((C + 63) / 64)), 0,
                       static_cast<hipStream_t>(hip_stream), ids, weight, rows, C, V, scale, out);
    return mtts::check_launch("embedding_fwd_kernel");
}

extern "C" int mtts_embedding_bwd(const int64_t *ids, const float *dout, int64_t rows, int32_t V, int32_t C,
                                  float scale, float *dweight, void *hip_stream) {
    MTTS_CHECK_ARG(ids && dout && dweight && rows >= 0 && V >= 1 && C >= 1 && rows <= 0x7fffffff,
                   "embedding_bwd: bad args");
    MTTS_CHECK_ARG(C <= 4 * kEThreads, "embedding_bwd: C > 1024");
    hipLaunchKernelGGL(embedding_bwd_kernel, dim3(V), dim3(kEThreads), 0, static_cast<hipStream_t>(hip_stream), ids,
                       dout, rows, C, scale, dweight);
    return mtts::check_launch("embedding_bwd_kernel");
}
