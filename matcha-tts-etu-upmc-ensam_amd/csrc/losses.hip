// Fused training losses of the Matcha-TTS step on gfx950:
//   diff_loss  = sum((u_pred - u)^2) / (sum(y_mask) * C),  u = x1 - (1 - sigma_min) * z  (UNMASKED, as
//                flow_matching.py:145-149: the padded frames contribute ((1 - sigma) z)^2)
//   prior_loss = sum(0.5 * ((y - mu_y)^2 + log(2 pi)) * y_mask) / (sum(y_mask) * C)   (matcha_tts.py:319-323)
// y_mask is the caller's float [B, T] frame mask (flow_matching.py's `mask`).
// and their backward (du_pred, dmu_y).  The reference's torch expression costs ~30 elementwise /
// reduction launches per step (sub, pow, mul, sum, div ... forward and backward); here: one partials
// kernel + one finalize kernel forward, one kernel backward.
//
// Layouts: u_pred / du_pred token-major [B, T, C] (the decoder's output layout); x1, z, y, mu_y, dmu_y
// channel-major [B, C, T].  One workgroup per (utterance, 64-frame tile): the token-major tile
// (64 x C contiguous floats) is staged through LDS (row pitch C+1: conflict-free transposed reads),
// the channel-major rows are read 64 frames at a time (256-byte coalesced).
// u = x1 - (1 - sigma) z rounds like torch's two ops (mul, then sub: built with -ffp-contract=off, the
// same as cfm_prep.hip's phi_t).
// Sums: per-thread fp32 in a fixed order, then a fixed tree per workgroup, then the finalize kernel
// sums the workgroup partials in index order -- deterministic and run-to-run identical.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "mtts_common.h"

namespace {

constexpr int kLT = 64;  // frames per workgroup
constexpr int kLThreads = 256;
constexpr int kLMaxC = 128;  // channels staged per tile
constexpr int kLPitch = kLMaxC + 1;

// Workgroup sum in a fixed order; the result is valid in thread 0.
__device__ __forceinline__ float block_sum(float v, float *red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float s = 0.f;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < kLThreads / 64; ++i) s += red[i];
    }
    return s;
}

__global__ __launch_bounds__(kLThreads) void loss_partials_kernel(const float *__restrict__ u_pred,
                                                                   const float *__restrict__ x1,
                                                                   const float *__restrict__ z,
                                                                   const float *__restrict__ y,
                                                                   const float *__restrict__ mu_y,
                                                                   const float *__restrict__ mask, int C,
                                                                   int T, float one_minus_sigma,
                                                                   float *__restrict__ partials) {
    __shared__ float su[kLT * kLPitch];
    __shared__ float red[kLThreads / 64];
    const int b = blockIdx.y, t0 = blockIdx.x * kLT;
    const int nt = min(kLT, T - t0);
    const float *mb = mask + (size_t)b * T + t0;
    const size_t cm = (size_t)b * C * T;  // channel-major utterance base
    float d_acc = 0.f, p_acc = 0.f;
    if (u_pred) {
        const float *ub = u_pred + ((size_t)b * T + t0) * C;
#pragma unroll 4
        for (int e = threadIdx.x; e < nt * C; e += kLThreads) {
            const int tl = e / C, c = e - tl * C;
            su[tl * kLPitch + c] = ub[e];
        }
        __syncthreads();
    }
#pragma unroll 4
    for (int e = threadIdx.x; e < C * kLT; e += kLThreads) {
        const int c = e / kLT, tl = e - c * kLT;
        if (tl >= nt) continue;
        const size_t i = cm + (size_t)c * T + t0 + tl;
        if (u_pred) {
            const float u = x1[i] - one_minus_sigma * z[i];
            const float d = su[tl * kLPitch + c] - u;
            d_acc = fmaf(d, d, d_acc);
        }
        if (mu_y) {
            const float d = y[i] - mu_y[i];
            p_acc += 0.5f * (d * d + 1.8378770664093453f) * mb[tl];  // log(2 pi)
        }
    }
    const float ds = block_sum(d_acc, red);
    const float ps = block_sum(p_acc, red);
    if (threadIdx.x == 0) {
        const size_t blk = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
        partials[2 * blk] = ds;
        partials[2 * blk + 1] = ps;
    }
}

__global__ __launch_bounds__(kLThreads) void loss_finalize_kernel(const float *__restrict__ partials, int nblk,
                                                                   const float *__restrict__ mask, int BT,
                                                                   int C, float *__restrict__ out) {
    __shared__ float red[kLThreads / 64];
    float d = 0.f, p = 0.f, m = 0.f;
    for (int i = threadIdx.x; i < nblk; i += kLThreads) {
        d += partials[2 * i];
        p += partials[2 * i + 1];
    }
    for (int i = threadIdx.x; i < BT; i += kLThreads) m += mask[i];
    d = block_sum(d, red);
    p = block_sum(p, red);
    m = block_sum(m, red);
    if (threadIdx.x == 0) {
        const float denom = m * (float)C;
        out[0] = d / denom;
        out[1] = p / denom;
        out[2] = denom;
    }
}

__global__ __launch_bounds__(kLThreads) void loss_bwd_kernel(const float *__restrict__ g_diff,
                                                              const float *__restrict__ g_prior,
                                                              const float *__restrict__ denom_p,
                                                              const float *__restrict__ u_pred,
                                                              const float *__restrict__ x1, const float *__restrict__ z,
                                                              const float *__restrict__ y,
                                                              const float *__restrict__ mu_y,
                                                              const float *__restrict__ mask, int C, int T,
                                                              float one_minus_sigma, float *__restrict__ du_pred,
                                                              float *__restrict__ dmu_y) {
    __shared__ float su[kLT * kLPitch];
    const int b = blockIdx.y, t0 = blockIdx.x * kLT;
    const int nt = min(kLT, T - t0);
    const float *mb = mask + (size_t)b * T + t0;
    const size_t cm = (size_t)b * C * T;
    const float denom = denom_p[0];
    if (du_pred) {
        // u (channel-major) -> LDS transposed, then du_pred written token-major, coalesced
    #pragma unroll 4
    for (int e = threadIdx.x; e < C * kLT; e += kLThreads) {
            const int c = e / kLT, tl = e - c * kLT;
            if (tl < nt) {
                const size_t i = cm + (size_t)c * T + t0 + tl;
                su[tl * kLPitch + c] = x1[i] - one_minus_sigma * z[i];
            }
        }
        __syncthreads();
        const float g = 2.f * g_diff[0] / denom;
        const size_t tb = ((size_t)b * T + t0) * C;
#pragma unroll 4
        for (int e = threadIdx.x; e < nt * C; e += kLThreads) {
            const int tl = e / C, c = e - tl * C;
            du_pred[tb + e] = g * (u_pred[tb + e] - su[tl * kLPitch + c]);
        }
    }
    if (dmu_y) {
        const float g = -g_prior[0] / denom;
    #pragma unroll 4
    for (int e = threadIdx.x; e < C * kLT; e += kLThreads) {
            const int c = e / kLT, tl = e - c * kLT;
            if (tl >= nt) continue;
            const size_t i = cm + (size_t)c * T + t0 + tl;
            dmu_y[i] = g * (y[i] - mu_y[i]) * mb[tl];
        }
    }
}

}  // namespace

extern "C" size_t mtts_losses_workspace_size(int32_t B, int32_t T) {
    if (B < 0 || T < 0) return 0;
    return (size_t)B * ((T + kLT - 1) / kLT) * 2 * sizeof(float);
}

extern "C" int mtts_losses_fwd(const float *u_pred, const float *x1, const float *z, const float *y,
                               const float *mu_y, const float *mask, int32_t B, int32_t C, int32_t T,
                               float sigma_min, float *out, void *workspace, size_t workspace_bytes,
                               void *hip_stream) {
    MTTS_CHECK_ARG(mask && out && B >= 1 && T >= 1 && C >= 1 && B <= 65535, "losses_fwd: bad args");
    MTTS_CHECK_ARG(C <= kLMaxC, "losses_fwd: C > 128");
    MTTS_CHECK_ARG(!u_pred || (x1 && z), "losses_fwd: the CFM loss needs x1 and z");
    MTTS_CHECK_ARG(!mu_y || y, "losses_fwd: the prior loss needs y");
    if (!workspace || workspace_bytes < mtts_losses_workspace_size(B, T))
        return mtts::fail(MTTS_ERR_WORKSPACE, "losses_fwd: workspace too small");
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    dim3 grid((T + kLT - 1) / kLT, B);
    float *part = static_cast<float *>(workspace);
    hipLaunchKernelGGL(loss_partials_kernel, grid, dim3(kLThreads), 0, st, u_pred, x1, z, y, mu_y, mask, C, T,
                       (float)(1.0 - (double)sigma_min), part);  // torch: (1 - s) is a Python double
    int rc = mtts::check_launch("loss_partials_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(kLThreads), 0, st, part, (int)(grid.x * grid.y), mask,
                       B * T, C, out);
    return mtts::check_launch("loss_finalize_kernel");
}

extern "C" int mtts_losses_bwd(const float *g_diff, const float *g_prior, const float *fwd_out, const float *u_pred, const float *x1,
                               const float *z, const float *y, const float *mu_y, const float *mask,
                               int32_t B, int32_t C, int32_t T, float sigma_min, float *du_pred, float *dmu_y,
                               void *hip_stream) {
    MTTS_CHECK_ARG(fwd_out && mask && B >= 1 && T >= 1 && C >= 1 && B <= 65535 && C <= kLMaxC,
                   "losses_bwd: bad args");
    MTTS_CHECK_ARG(!du_pred || (g_diff && u_pred && x1 && z), "losses_bwd: du_pred needs g_diff, u_pred, x1, z");
    MTTS_CHECK_ARG(!dmu_y || (g_prior && y && mu_y), "losses_bwd: dmu_y needs g_prior, y, mu_y");
    if (!du_pred && !dmu_y) return MTTS_OK;
    dim3 grid((T + kLT - 1) / kLT, B);
    hipLaunchKernelGGL(loss_bwd_kernel, grid, dim3(kLThreads), 0, static_cast<hipStream_t>(hip_stream), g_diff,
                       g_prior, fwd_out + 2, u_pred, x1, z, y, mu_y, mask, C, T, (float)(1.0 - (double)sigma_min), du_pred,
                       dmu_y);
    return mtts::check_launch("loss_bwd_kernel");
}

// ------------------------------------------------------------------------------------------------
// Step glue (matcha_tts.py:259-288, model.py:13-34 / 117-135, text_encoder.py:398 / 300-303):
//   sequence masks from the lengths (0/1 fp32, and the text encoder's -1e4 key bias), the duration loss
//     logw_ = log(1e-8 + dur) * x_mask ;  dur_loss = sum((logw - logw_)^2) / sum(x_lengths)
//   with its backward, and the step's loss sum + logged vector.  Each used to be a chain of 3..10 tiny
//   torch launches (arange / lt / cast, add / log / mul / sub / pow / sum / sum / div, add / add / stack).
// Roundings follow torch's op sequence (-ffp-contract=off): (1e-8f + dur), logf, * mask, -, d * d;
// the sums run in a fixed order (deterministic; torch's tree order differs by an ulp).
namespace {

constexpr int kGThreads = 1024;

__global__ __launch_bounds__(256) void sequence_mask_kernel(const int64_t *__restrict__ lengths, int B, int T,
                                                            float *__restrict__ mask, float *__restrict__ key_bias) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)B * T) return;
    const int b = (int)(i / T), t = (int)(i - (int64_t)b * T);
    const float m = (int64_t)t < lengths[b] ? 1.f : 0.f;
    if (mask) mask[i] = m;
    if (key_bias) key_bias[i] = (m - 1.0f) * 1e4f;
}

__device__ __forceinline__ float big_block_sum(float v, float *red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float s = 0.f;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < kGThreads / 64; ++i) s += red[i];
    }
    return s;
}

__device__ __forceinline__ float dur_diff(const float *logw, const float *dur, const int64_t *lengths, int T, int64_t i) {
    const int b = (int)(i / T), t = (int)(i - (int64_t)b * T);
    const float m = (int64_t)t < lengths[b] ? 1.f : 0.f;
    const float target = logf(1e-8f + dur[i]) * m;
    return logw[i] - target;
}

// one workgroup: B*T is the text side (a few thousand entries)
__global__ __launch_bounds__(kGThreads) void duration_loss_fwd_kernel(const float *__restrict__ logw,
                                                                      const float *__restrict__ dur,
                                                                      const int64_t *__restrict__ lengths, int B, int T,
                                                                      float *__restrict__ out) {
    __shared__ float red[kGThreads / 64];
    float acc = 0.f;
    for (int64_t i = threadIdx.x; i < (int64_t)B * T; i += kGThreads) {
        const float d = dur_diff(logw, dur, lengths, T, i);
        acc += d * d;
    }
    const float s = big_block_sum(acc, red);
    if (threadIdx.x == 0) {
        int64_t l = 0;
        for (int b = 0; b < B; ++b) l += lengths[b];
        const float L = (float)l;  // torch: float32 / int64 -> float32
        out[0] = s / L;
        out[1] = L;
    }
}

__global__ __launch_bounds__(256) void duration_loss_bwd_kernel(const float *__restrict__ g,
                                                                const float *__restrict__ fwd_out,
                                                                const float *__restrict__ logw,
                                                                const float *__restrict__ dur,
                                                                const int64_t *__restrict__ lengths, int B, int T,
                                                                float *__restrict__ dlogw) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)B * T) return;
    const float gl = g[0] / fwd_out[1];  // DivBackward: grad / sum(lengths)
    const float d = dur_diff(logw, dur, lengths, T, i);
    dlogw[i] = gl * (2.0f * d);  // PowBackward (exponent 2): grad * (2 * d)
}

// total = (dur + prior) + diff (torch's left-to-right adds); logged = [dur, prior, diff, total]
__global__ void loss_sum_kernel(const float *__restrict__ dur, const float *__restrict__ prior,
                                const float *__restrict__ diff, float *__restrict__ total, float *__restrict__ logged) {
    if (threadIdx.x != 0) return;
    const float d = dur[0], p = prior ? prior[0] : 0.f, f = diff[0];
    const float t = (d + p) + f;
    total[0] = t;
    if (logged) {
        logged[0] = d;
        logged[1] = p;
        logged[2] = f;
        logged[3] = t;
    }
}

}  // namespace

extern "C" int mtts_sequence_mask_f32(const int64_t *lengths, int32_t B, int32_t T, float *mask, float *key_bias,
                                      void *hip_stream) {
    MTTS_CHECK_ARG(lengths && B >= 0 && T >= 0 && (mask || key_bias), "sequence_mask_f32: bad args");
    const int64_t n = (int64_t)B * T;
    if (n == 0) return MTTS_OK;
    hipLaunchKernelGGL(sequence_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(hip_stream), lengths, B, T, mask, key_bias);
    return mtts::check_launch("sequence_mask_kernel");
}

extern "C" int mtts_duration_loss_fwd(const float *logw, const float *dur, const int64_t *lengths, int32_t B, int32_t T,
                                      float *out, void *hip_stream) {
    MTTS_CHECK_ARG(logw && dur && lengths && out && B >= 1 && T >= 1, "duration_loss_fwd: bad args");
    hipLaunchKernelGGL(duration_loss_fwd_kernel, dim3(1), dim3(kGThreads), 0, static_cast<hipStream_t>(hip_stream),
                       logw, dur, lengths, B, T, out);
    return mtts::check_launch("duration_loss_fwd_kernel");
}

extern "C" int mtts_duration_loss_bwd(const float *g, const float *fwd_out, const float *logw, const float *dur,
                                      const int64_t *lengths, int32_t B, int32_t T, float *dlogw, void *hip_stream) {
    MTTS_CHECK_ARG(g && fwd_out && logw && dur && lengths && dlogw && B >= 1 && T >= 1, "duration_loss_bwd: bad args");
    const int64_t n = (int64_t)B * T;
    hipLaunchKernelGGL(duration_loss_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(hip_stream), g, fwd_out, logw, dur, lengths, B, T, dlogw);
    return mtts::check_launch("duration_loss_bwd_kernel");
}

extern "C" int mtts_loss_sum(const float *dur, const float *prior, const float *diff, float *total, float *logged,
                             void *hip_stream) {
    MTTS_CHECK_ARG(dur && diff && total, "loss_sum: bad args");
    hipLaunchKernelGGL(loss_sum_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(hip_stream), dur, prior, diff,
                       total, logged);
    return mtts::check_launch("loss_sum_kernel");
}
