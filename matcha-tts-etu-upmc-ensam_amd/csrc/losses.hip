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
        for (int e = threadIdx.x; e < nt * C; e += kLThreads) {
            const int tl = e / C, c = e - tl * C;
            su[tl * kLPitch + c] = ub[e];
        }
        __syncthreads();
    }
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
        for (int e = threadIdx.x; e < nt * C; e += kLThreads) {
            const int tl = e / C, c = e - tl * C;
            du_pred[tb + e] = g * (u_pred[tb + e] - su[tl * kLPitch + c]);
        }
    }
    if (dmu_y) {
        const float g = -g_prior[0] / denom;
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
