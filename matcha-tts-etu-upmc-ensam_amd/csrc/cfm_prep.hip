// Decoder-input preparation of the CFM training step on gfx950 (reference: flow_matching.py:130-145 and
// decoder.py:8-31, 288):
//   mtts_cfm_pack_fwd : phi_t = (1 - (1 - sigma) t) z + t x1 (flow_matching.py:138) and the channel
//                       concat with mu (decoder.py:288, einops pack), written straight into the decoder's
//                       token-major input [B, T, 2C] = [phi^T | mu^T] -- one pass instead of the scalar
//                       ops on t, two multiplies, an add, two transposes and a concat.
//   mtts_cfm_pack_bwd : the gradient of mu from that input (d_mu = d_packed[..., C:]^T), one transpose.
//   mtts_time_embedding: SinusoidalPosEmb (decoder.py:8-31) in one launch instead of arange / mul / exp /
//                       mul / mul / sin / cos / cat.
// Arithmetic follows torch's elementwise order exactly (separate fp32 roundings, no contraction:
// __fmul_rn / __fadd_rn / __fsub_rn), so phi and the embedding equal the torch expressions bit for bit
// up to the device libm's expf / sinf / cosf, which torch's kernels also call.
// Layout: one workgroup per (utterance, 32-frame tile); channel-major rows are read 32 frames at a
// time (128-byte coalesced), staged in LDS (pitch 33: conflict-free transposed reads), and written as
// contiguous token-major rows.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "mtts_common.h"

namespace {

constexpr int kPT = 32;  // frames per workgroup (B=32 x 600 frames: 608 workgroups, 33 KB LDS each)
constexpr int kPThreads = 256;
constexpr int kPMaxC = 128;
constexpr int kPPitch = kPT + 1;

__global__ __launch_bounds__(kPThreads) void cfm_pack_fwd_kernel(const float *__restrict__ x1,
                                                                  const float *__restrict__ z,
                                                                  const float *__restrict__ t,
                                                                  const float *__restrict__ mu, int C, int T,
                                                                  float one_minus_sigma,
                                                                  float *__restrict__ packed) {
    __shared__ float sphi[kPMaxC * kPPitch];
    __shared__ float smu[kPMaxC * kPPitch];
    const int b = blockIdx.y, t0 = blockIdx.x * kPT;
    const int nt = min(kPT, T - t0);
    const float tb = t[b];
    const float a = __fsub_rn(1.f, __fmul_rn(one_minus_sigma, tb));  // 1 - (1 - s) * t
    const size_t cm = (size_t)b * C * T + t0;
    for (int e = threadIdx.x; e < C * kPT; e += kPThreads) {
        const int c = e / kPT, tl = e - c * kPT;
        if (tl < nt) {
            const size_t i = cm + (size_t)c * T + tl;
            sphi[c * kPPitch + tl] = __fadd_rn(__fmul_rn(a, z[i]), __fmul_rn(tb, x1[i]));
            smu[c * kPPitch + tl] = mu[i];
        }
    }
    __syncthreads();
    const int C2 = 2 * C;
    float *ob = packed + ((size_t)b * T + t0) * C2;
    for (int e = threadIdx.x; e < nt * C2; e += kPThreads) {
        const int tl = e / C2, c = e - tl * C2;
        ob[e] = c < C ? sphi[c * kPPitch + tl] : smu[(c - C) * kPPitch + tl];
    }
}

__global__ __launch_bounds__(kPThreads) void cfm_pack_bwd_kernel(const float *__restrict__ d_packed, int C, int T,
                                                                  float *__restrict__ d_mu) {
    __shared__ float s[kPT * (kPMaxC + 1)];
    const int b = blockIdx.y, t0 = blockIdx.x * kPT;
    const int nt = min(kPT, T - t0);
    const int C2 = 2 * C;
    const float *ib = d_packed + ((size_t)b * T + t0) * C2 + C;
    for (int e = threadIdx.x; e < nt * C; e += kPThreads) {
        const int tl = e / C, c = e - tl * C;
        s[tl * (kPMaxC + 1) + c] = ib[(size_t)tl * C2 + c];
    }
    __syncthreads();
    const size_t cm = (size_t)b * C * T + t0;
    for (int e = threadIdx.x; e < C * kPT; e += kPThreads) {
        const int c = e / kPT, tl = e - c * kPT;
        if (tl < nt) d_mu[cm + (size_t)c * T + tl] = s[tl * (kPMaxC + 1) + c];
    }
}

__global__ __launch_bounds__(256) void time_embedding_kernel(const float *__restrict__ t, int half, float neg_step,
                                                              float scale, float *__restrict__ out) {
    const int b = blockIdx.x;
    const float st = __fmul_rn(scale, t[b]);  // scale * x
    for (int k = threadIdx.x; k < half; k += 256) {
        const float freq = expf(__fmul_rn((float)k, neg_step));  // exp(arange * -step)
        const float arg = __fmul_rn(st, freq);
        out[(size_t)b * 2 * half + k] = sinf(arg);
        out[(size_t)b * 2 * half + half + k] = cosf(arg);
    }
}

}  // namespace

extern "C" int mtts_cfm_pack_fwd(const float *x1, const float *z, const float *t, const float *mu, int32_t B,
                                 int32_t C, int32_t T, float sigma_min, float *packed, void *hip_stream) {
    MTTS_CHECK_ARG(x1 && z && t && mu && packed, "cfm_pack_fwd: null pointer");
    MTTS_CHECK_ARG(B >= 0 && B <= 65535 && C >= 1 && C <= kPMaxC && T >= 0, "cfm_pack_fwd: bad shape (C <= 128)");
    if ((size_t)B * T == 0) return MTTS_OK;
    dim3 grid((T + kPT - 1) / kPT, B);
    hipLaunchKernelGGL(cfm_pack_fwd_kernel, grid, dim3(kPThreads), 0, static_cast<hipStream_t>(hip_stream), x1, z, t,
                       mu, C, T, (float)(1.0 - (double)sigma_min), packed);  // torch: (1 - s) is a Python double
    return mtts::check_launch("cfm_pack_fwd_kernel");
}

extern "C" int mtts_cfm_pack_bwd(const float *d_packed, int32_t B, int32_t C, int32_t T, float *d_mu,
                                 void *hip_stream) {
    MTTS_CHECK_ARG(d_packed && d_mu, "cfm_pack_bwd: null pointer");
    MTTS_CHECK_ARG(B >= 0 && B <= 65535 && C >= 1 && C <= kPMaxC && T >= 0, "cfm_pack_bwd: bad shape (C <= 128)");
    if ((size_t)B * T == 0) return MTTS_OK;
    dim3 grid((T + kPT - 1) / kPT, B);
    hipLaunchKernelGGL(cfm_pack_bwd_kernel, grid, dim3(kPThreads), 0, static_cast<hipStream_t>(hip_stream), d_packed,
                       C, T, d_mu);
    return mtts::check_launch("cfm_pack_bwd_kernel");
}

extern "C" int mtts_time_embedding(const float *t, int32_t B, int32_t dim, float scale, float *out,
                                   void *hip_stream) {
    MTTS_CHECK_ARG(t && out && B >= 0 && dim >= 4 && dim % 2 == 0, "time_embedding: bad args (dim even, >= 4)");
    if (B == 0) return MTTS_OK;
    const int half = dim / 2;
    const float neg_step = -(float)(std::log(10000.0) / (half - 1));  // torch: arange * -step, step a Python float
    hipLaunchKernelGGL(time_embedding_kernel, dim3(B), dim3(256), 0, static_cast<hipStream_t>(hip_stream), t, half,
                       neg_step, scale, out);
    return mtts::check_launch("time_embedding_kernel");
}
