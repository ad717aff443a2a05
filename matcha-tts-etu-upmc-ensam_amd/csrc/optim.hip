// Gradient-norm clipping + AdamW over every parameter of the model in two launches (gfx950).
//
// Reference step semantics (train.py:81-102 -> Lightning: gradient_clip_val=1.0, norm-2 clipping
// over all parameters; baselightningmodule.py:59-65: AdamW(lr, betas=(0.9, 0.999), weight_decay=1e-6,
// eps=1e-8)), i.e. torch.nn.utils.clip_grad_norm_ followed by torch.optim.AdamW:
//   total = ||g||_2 over all parameters,  coef = min(max_norm / (total + 1e-6), 1)
//   g' = g * coef;  p *= 1 - lr*wd;  m = m + (1-b1)(g' - m);  v = b2 v + (1-b2) g'^2
//   p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// with torch's scalars (double on the host, rounded to fp32 once) and one rounding per torch op, so
// the result is within 1-2 ulp of torch's AdamW (tests/test_training_gpu.py).
// torch runs this as ~8 multi-tensor launches (norm, scale, fused Adam per dtype/device group) over
// ~300 tensors: 0.44 ms per step at 19 M parameters.  Here the parameters and both moment buffers
// are one flat fp32 array each (the model's parameters are views into it), the gradients are
// addressed through a chunk table (gradients stay wherever autograd put them), and
//   adamw_sumsq_kernel   one block per chunk: partial sum of squares (fixed order); block 0 also
//                        stages t + 1 of the device step counter
//   adamw_update_kernel  one block per chunk: every block sums all partials in the same fixed order
//                        (deterministic, no grid barrier), clips and updates its chunk; block 0
//                        stores the new step count (read by no block of this launch: no race).
// Everything, the step count and the learning rate included, stays on the device: the pair of
// launches is replayed as is inside a HIP graph.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float block_reduce_sum(float v, float *red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kThreads / 64; ++i) s += red[i];
    return s;
}

__global__ __launch_bounds__(kThreads) void adamw_sumsq_kernel(const mtts_adamw_chunk *__restrict__ chunks,
                                                               float *__restrict__ partial, const float *__restrict__ step,
                                                               float *__restrict__ t_next) {
    __shared__ float red[kThreads / 64];
    if (blockIdx.x == 0 && threadIdx.x == 0) t_next[0] = step[0] + 1.f;
    const mtts_adamw_chunk c = chunks[blockIdx.x];
    // The summation order depends on the chunk's values only, never on where its gradient lives: the
    // data-parallel step keeps gradients in bucket views whose alignment differs from the allocator's,
    // and both must clip with the same norm bit for bit.  Thread t sums groups of 4 (t, t + 256, ...);
    // an unaligned or ragged group is loaded element-wise with zeros past the end.
    // (kU groups are loaded before any is summed -- kU loads in flight per thread -- and summed in the
    // same order as one group at a time)
    float s = 0.f;
    const bool vec = ((uintptr_t)c.grad & 15) == 0;
    const int ng = (c.n + 3) / 4;
    auto load = [&](int i) {
        if (i >= ng) return make_float4(0.f, 0.f, 0.f, 0.f);
        if (vec && 4 * i + 4 <= c.n) return reinterpret_cast<const float4 *>(c.grad)[i];
        const float *q = c.grad + 4 * i;
        const int r = c.n - 4 * i;
        return make_float4(q[0], r > 1 ? q[1] : 0.f, r > 2 ? q[2] : 0.f, r > 3 ? q[3] : 0.f);
    };
    constexpr int kU = 4;
    for (int i0 = threadIdx.x; i0 < ng; i0 += kU * kThreads) {
        float4 g[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) g[u] = load(i0 + u * kThreads);
#pragma unroll
        for (int u = 0; u < kU; ++u)
            if (i0 + u * kThreads < ng) s += (g[u].x * g[u].x + g[u].y * g[u].y) + (g[u].z * g[u].z + g[u].w * g[u].w);
    }
    s = block_reduce_sum(s, red);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(kThreads) void adamw_update_kernel(const mtts_adamw_chunk *__restrict__ chunks, int nchunks,
                                                                const float *__restrict__ partial, float *__restrict__ p,
                                                                float *__restrict__ m, float *__restrict__ v,
                                                                const double *__restrict__ lr_ptr,
                                                                const float *__restrict__ t_next,
                                                                float *__restrict__ step, float max_norm, double b1,
                                                                double b2, double eps_d, double wd, float gscale) {
    __shared__ float red[kThreads / 64];
    // total squared norm: every block sums the same partials in the same order
    float s = 0.f;
    for (int i = threadIdx.x; i < nchunks; i += kThreads) s += partial[i];
    // (the partials are sums of the raw g^2; g * gscale has norm sqrt(sum g^2) * gscale -- the same fp32
    // value for a power-of-two gscale, which scales exactly)
    const float total = sqrtf(block_reduce_sum(s, red)) * gscale;
    // clip_grad_norm_: coef = clamp(max_norm / (total + 1e-6), max=1), fp32 tensor arithmetic
    float coef = 1.f;
    if (max_norm > 0.f) coef = fminf(max_norm / (total + 1e-6f), 1.f);
    const float t = t_next[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) step[0] = t;
    // torch's multi-tensor AdamW (torch/optim/adam.py, decoupled weight decay) derives every scalar in
    // double precision on the host and hands it to fp32 kernels: the same here, so each constant is the
    // float torch uses (computing 1 - b2 from a float b2 would be off by 1.3e-5 relative)
    const double lr = lr_ptr[0];
    const float decay = (float)(1.0 - lr * wd);
    const float w1 = (float)(1.0 - b1), b2f = (float)b2, w2 = (float)(1.0 - b2);
    const float neg_step = (float)(-(lr / (1.0 - pow(b1, (double)t))));
    const float bc2s = (float)sqrt(1.0 - pow(b2, (double)t));
    const float eps = (float)eps_d;
    const mtts_adamw_chunk c = chunks[blockIdx.x];
    float *pp = p + c.offset, *mm = m + c.offset, *vv = v + c.offset;
    // one fp32 rounding per torch op: _foreach_mul_(grads, coef), _foreach_mul_(params, 1 - lr wd),
    // _foreach_lerp_(m, g, 1 - b1) (weight < 0.5: m + w (g - m)), _foreach_mul_(v, b2),
    // _foreach_addcmul_(v, g, g, 1 - b2), sqrt(v) / sqrt(bc2) + eps, _foreach_addcdiv_(p, m, denom, -lr / bc1)
    auto upd = [&](float g, float &pi, float &mi, float &vi) {
        g = __fmul_rn(__fmul_rn(g, gscale), coef);
        pi = __fmul_rn(pi, decay);
        mi = __fadd_rn(mi, __fmul_rn(w1, __fsub_rn(g, mi)));
        vi = __fmul_rn(vi, b2f);
        vi = __fadd_rn(vi, __fmul_rn(__fmul_rn(w2, g), g));
        const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(vi), bc2s), eps);
        pi = __fadd_rn(pi, __fmul_rn(neg_step, __fdiv_rn(mi, denom)));
    };
    const bool vec = (((uintptr_t)c.grad | (uintptr_t)pp) & 15) == 0;  // flat regions start 16-byte aligned
    const int n4 = vec ? c.n / 4 : 0;
    // two float4 groups per thread per iteration, all eight loads issued first (one group at a time kept
    // ~4 KB in flight per wave: 110 us for the 532 MB the update streams)
    constexpr int kU = 2;
    for (int i0 = threadIdx.x; i0 < n4; i0 += kU * kThreads) {
        float4 g[kU], a[kU], b[kU], d[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int i = i0 + u * kThreads;
            if (i < n4) {
                g[u] = reinterpret_cast<const float4 *>(c.grad)[i];
                a[u] = reinterpret_cast<float4 *>(pp)[i];
                b[u] = reinterpret_cast<float4 *>(mm)[i];
                d[u] = reinterpret_cast<float4 *>(vv)[i];
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int i = i0 + u * kThreads;
            if (i < n4) {
                upd(g[u].x, a[u].x, b[u].x, d[u].x);
                upd(g[u].y, a[u].y, b[u].y, d[u].y);
                upd(g[u].z, a[u].z, b[u].z, d[u].z);
                upd(g[u].w, a[u].w, b[u].w, d[u].w);
                reinterpret_cast<float4 *>(pp)[i] = a[u];
                reinterpret_cast<float4 *>(mm)[i] = b[u];
                reinterpret_cast<float4 *>(vv)[i] = d[u];
            }
        }
    }
    for (int i = 4 * n4 + threadIdx.x; i < c.n; i += kThreads) upd(c.grad[i], pp[i], mm[i], vv[i]);
}

}  // namespace

extern "C" size_t mtts_clip_adamw_workspace_size(int32_t nchunks) {
    return (size_t)(nchunks > 0 ? nchunks + 1 : 0) * sizeof(float);
}

extern "C" int mtts_clip_adamw_scaled(const mtts_adamw_chunk *chunks, int32_t nchunks, float *params,
                                      float *exp_avg, float *exp_avg_sq, const double *lr, float *step, float max_norm,
                                      double beta1, double beta2, double eps, double weight_decay, float grad_scale,
                                      void *workspace, size_t workspace_bytes, void *hip_stream) {
    MTTS_CHECK_ARG(chunks && params && exp_avg && exp_avg_sq && lr && step && nchunks >= 0,
                   "clip_adamw: null pointer");
    MTTS_CHECK_ARG(grad_scale > 0.f, "clip_adamw: grad_scale must be positive");
    if (nchunks == 0) return MTTS_OK;
    if (!workspace || workspace_bytes < mtts_clip_adamw_workspace_size(nchunks))
        return mtts::fail(MTTS_ERR_WORKSPACE, "clip_adamw: workspace too small");
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    float *partial = static_cast<float *>(workspace), *t_next = partial + nchunks;
    hipLaunchKernelGGL(adamw_sumsq_kernel, dim3(nchunks), dim3(kThreads), 0, st, chunks, partial, (const float *)step,
                       t_next);
    int rc = mtts::check_launch("adamw_sumsq_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(adamw_update_kernel, dim3(nchunks), dim3(kThreads), 0, st, chunks, nchunks,
                       (const float *)partial, params, exp_avg, exp_avg_sq, lr, (const float *)t_next, step, max_norm,
                       beta1, beta2, eps, weight_decay, grad_scale);
    return mtts::check_launch("adamw_update_kernel");
}

extern "C" int mtts_clip_adamw(const mtts_adamw_chunk *chunks, int32_t nchunks, float *params, float *exp_avg,
                               float *exp_avg_sq, const double *lr, float *step, float max_norm, double beta1,
                               double beta2, double eps, double weight_decay, void *workspace,
                               size_t workspace_bytes, void *hip_stream) {
    return mtts_clip_adamw_scaled(chunks, nchunks, params, exp_avg, exp_avg_sq, lr, step, max_norm, beta1, beta2, eps,
                                  weight_decay, 1.0f, workspace, workspace_bytes, hip_stream);
}
