// Token embedding of the text encoder (text_encoder.py:341-342, :389):
//   out[r, :] = W[ids[r], :] * scale            (nn.Embedding lookup, then * sqrt(C))
// and its weight gradient
//   dW[v, :] = sum over rows r with ids[r] == v of (dout[r, :] * scale)
// torch's embedding backward on the GPU sums with atomics (a run-to-run varying order); here the
// workgroups of vocabulary entry v sum its rows in a fixed order, so the gradient is deterministic and
// the whole training step bit-reproducible.  Each term is rounded as torch rounds it (the scale
// product first, then the sum): -ffp-contract is irrelevant, the product and sum are separate ops.
//
// ids are read V x C/64 times from L2 (8 B x rows each: 14 MB at B=32, Tx=120, V=150, C=192), dout
// once.
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
    const int64_t v = ids[r];
    float *dst = out + r * C;
    if (v < 0 || v >= V) {
        // nn.Embedding raises a device-side assert on an out-of-range id; a stream-ordered kernel cannot
        // raise, so the row is poisoned with NaN instead: the losses turn NaN at once, never silently
        // training on a clamped entry (collate() validates ids on the host as well)
        for (int c = threadIdx.x; c < C; c += blockDim.x) dst[c] = __builtin_nanf("");
        return;
    }
    const float *src = w + v * C;
    for (int c = threadIdx.x; c < C; c += blockDim.x) dst[c] = src[c] * scale;
}

// One workgroup per (vocabulary entry v, 64-channel slice): the ids are scanned 1024 rows at a time,
// the rows holding v compacted into LDS in ascending row order (wave ballots + popcount prefixes),
// then wave w sums the compacted rows k = w, w + 4, ... (four loads in flight per lane), and the four
// wave partials are added in wave order.  A token owning hundreds of rows (the padding id) is summed
// by 4 waves x 4 loads in flight instead of one dependent chain.
constexpr int kEChunk = 4 * kEThreads;

__global__ __launch_bounds__(kEThreads) void embedding_bwd_kernel(const int64_t *__restrict__ ids,
                                                                   const float *__restrict__ dout, int64_t rows,
                                                                   int C, float scale, float *__restrict__ dw) {
    __shared__ int s_rows[kEChunk];
    __shared__ int s_cnt[4][kEThreads / 64];
    __shared__ float s_part[kEThreads / 64][64];
    const int v = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = blockIdx.y * 64 + lane;
    const bool cok = c < C;
    float acc = 0.f;
    for (int64_t r0 = 0; r0 < rows; r0 += kEChunk) {
        uint64_t m[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // sub-chunk j covers rows r0 + 256 j + tid
            const int64_t r = r0 + j * kEThreads + threadIdx.x;
            m[j] = __ballot(r < rows && ids[r] == v);
            if (lane == 0) s_cnt[j][wave] = __popcll(m[j]);
        }
        __syncthreads();
        int total = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int base = total;
#pragma unroll
            for (int w = 0; w < kEThreads / 64; ++w) {
                base += w < wave ? s_cnt[j][w] : 0;
                total += s_cnt[j][w];
            }
            if ((m[j] >> lane) & 1ull)
                s_rows[base + __popcll(m[j] & ((1ull << lane) - 1ull))] = j * kEThreads + threadIdx.x;
        }
        __syncthreads();
        const float *src = dout + r0 * C + c;
        int k = wave;
        for (; k + 12 < total; k += 16) {  // four independent loads, added in k order
            const float a0 = cok ? src[(int64_t)s_rows[k] * C] : 0.f;
            const float a1 = cok ? src[(int64_t)s_rows[k + 4] * C] : 0.f;
            const float a2 = cok ? src[(int64_t)s_rows[k + 8] * C] : 0.f;
            const float a3 = cok ? src[(int64_t)s_rows[k + 12] * C] : 0.f;
            acc += a0 * scale;
            acc += a1 * scale;
            acc += a2 * scale;
            acc += a3 * scale;
        }
        for (; k < total; k += 4) acc += (cok ? src[(int64_t)s_rows[k] * C] : 0.f) * scale;
        __syncthreads();  // s_rows / s_cnt are rewritten by the next chunk
    }
    s_part[wave][lane] = acc;
    __syncthreads();
    if (wave == 0 && cok) dw[(int64_t)v * C + c] = ((s_part[0][lane] + s_part[1][lane]) + s_part[2][lane]) + s_part[3][lane];
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
    hipLaunchKernelGGL(embedding_bwd_kernel, dim3(V, (C + 63) / 64), dim3(kEThreads), 0,
                       static_cast<hipStream_t>(hip_stream), ids, dout, rows, C, scale, dweight);
    return mtts::check_launch("embedding_bwd_kernel");
}
