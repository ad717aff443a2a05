// Fused normalisation kernels of the CFM decoder, token-major [B*T, C] fp32 (gfx950).
//
// gn_mish_*: Block1D tail  mish(GroupNorm(conv)) * mask  (decoder.py:58-66), with Resnet1D's
//            time-embedding add (decoder.py:82-83) fused; one workgroup per (batch, group), the group's
//            T x C/G values stay in L1/L2 across the three passes (mean, centred variance, apply).
//            Backward recomputes xhat / mish' from h and the saved statistics; per-(b, c) partial
//            gamma/beta sums and the time-bias gradient come out of the same pass, and the gamma/beta
//            partials are reduced over the batch in a fixed order by reduce.hip (deterministic, batchable).
// layernorm_*: one wave per token row (norm1 / norm3 of BasicTransformerBlock, transformer.py:316,345).
// Numerics follow torch: mish(x) = x * tanh(log1p(exp(x))), two-pass variance, biased, eps inside sqrt.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

constexpr int kThreads = 256;

// mish(x) = x * tanh(softplus(x)) with ONE exponential: for e = exp(x), tanh(log(1 + e)) =
// ((1+e)^2 - 1) / ((1+e)^2 + 1) = n / (n + 2), n = e (e + 2); sigmoid(x) = e / (1 + e).  x is clamped at
// 15 (tanh(softplus(15)) rounds to 1 in fp32) so n never overflows.  Agrees with torch's
// x * tanh(log1p(exp(x))) to a few ulp; the three-transcendental form made the GroupNorm backward
// VALU-bound.
__device__ __forceinline__ float tanh_softplus(float x, float &sig) {
    const float e = __expf(fminf(x, 15.f));
    const float n = e * (e + 2.f);
    sig = e / (1.f + e);
    return n / (n + 2.f);
}

__device__ __forceinline__ float mish_f(float x) {
    float sig;
    return x * tanh_softplus(x, sig);
}

__device__ __forceinline__ float mish_grad(float x) {
    float sig;
    const float tsp = tanh_softplus(x, sig);
    return tsp + x * sig * (1.f - tsp * tsp);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// block-wide sum over NT threads, result broadcast to all threads (fixed reduction order)
template <int NT = kThreads>
__device__ __forceinline__ float block_sum(float v, float *red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) s += red[i];
    return s;
}

// 4 consecutive elements of an fp32 or bf16 tensor (bf16 -> fp32 is exact), and the store back (one
// rounding to bf16, v_cvt_pk_bf16_f32)
template <typename T>
__device__ __forceinline__ float4 ld4(const T *p) {
    if constexpr (sizeof(T) == 4) {
        return *reinterpret_cast<const float4 *>(p);
    } else {
        const uint2 q = *reinterpret_cast<const uint2 *>(p);
        return make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                           __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u));
    }
}

template <typename T>
__device__ __forceinline__ void st4(T *p, float4 v) {
    if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<float4 *>(p) = v;
    } else {
        typedef float f2 __attribute__((ext_vector_type(2)));
        typedef __bf16 h2 __attribute__((ext_vector_type(2)));
        const uint32_t lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){v.x, v.y}, h2));
        const uint32_t hi = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){v.z, v.w}, h2));
        *reinterpret_cast<uint2 *>(p) = make_uint2(lo, hi);
    }
}

// GroupNorm kernels: one 16-wave workgroup per (batch, group), so the three streaming passes over
// the group's T x C/G values keep enough loads in flight (256 workgroups fill the 256 CUs)
constexpr int kGnThreads = 1024;

// thread layout inside a group: cg/4 float4 columns, kThreads/(cg/4) token rows per pass
// TH / TY: storage of h / y (float, or uint16_t = bf16 bits: MTTS_NORM_F_X_BF16 / _Y_BF16)
template <typename TH, typename TY>
__global__ __launch_bounds__(kGnThreads) void gn_mish_fwd_kernel(const TH *__restrict__ h, const float *__restrict__ gamma,
                                                               const float *__restrict__ beta,
                                                               const float *__restrict__ mask,
                                                               const float *__restrict__ add, TY *__restrict__ y,
                                                               float *__restrict__ mean_out,
                                                               float *__restrict__ rstd_out, int T, int C, int G,
                                                               float eps) {
    __shared__ float red[kGnThreads / 64];
    const int g = blockIdx.x, b = blockIdx.y;
    const int cg = C / G;
    const int cols = cg / 4;
    const int rows_per_pass = kGnThreads / cols;
    const int tid = threadIdx.x;
    const int col = tid % cols, r0 = tid / cols;
    const bool active = r0 < rows_per_pass;
    const int c0 = g * cg + col * 4;
    const TH *hb = h + (size_t)b * T * C + c0;
    const float n = (float)T * cg;

    float s = 0.f;
    if (active)
        for (int t = r0; t < T; t += rows_per_pass) {
            const float4 v = ld4(hb + (size_t)t * C);
            s += (v.x + v.y) + (v.z + v.w);
        }
    const float mean = block_sum<kGnThreads>(s, red) / n;
    float q = 0.f;
    if (active)
        for (int t = r0; t < T; t += rows_per_pass) {
            const float4 v = ld4(hb + (size_t)t * C);
            const float a = v.x - mean, bq = v.y - mean, cq = v.z - mean, d = v.w - mean;
            q += (a * a + bq * bq) + (cq * cq + d * d);
        }
    const float var = block_sum<kGnThreads>(q, red) / n;
    const float rstd = rsqrtf(var + eps);
    if (tid == 0) {
        mean_out[b * G + g] = mean;
        rstd_out[b * G + g] = rstd;
    }
    if (!active) return;
    const float4 ga = *reinterpret_cast<const float4 *>(gamma + c0);
    const float4 be = *reinterpret_cast<const float4 *>(beta + c0);
    float4 ad = make_float4(0.f, 0.f, 0.f, 0.f);
    if (add) ad = *reinterpret_cast<const float4 *>(add + (size_t)b * C + c0);
    TY *yb = y + (size_t)b * T * C + c0;
    for (int t = r0; t < T; t += rows_per_pass) {
        const float4 v = ld4(hb + (size_t)t * C);
        const float m = mask ? mask[(size_t)b * T + t] : 1.f;
        float4 o;
        o.x = mish_f((v.x - mean) * rstd * ga.x + be.x) * m + ad.x;
        o.y = mish_f((v.y - mean) * rstd * ga.y + be.y) * m + ad.y;
        o.z = mish_f((v.z - mean) * rstd * ga.z + be.z) * m + ad.z;
        o.w = mish_f((v.w - mean) * rstd * ga.w + be.w) * m + ad.w;
        st4(yb + (size_t)t * C, o);
    }
}

// Per-channel partials of the GroupNorm backward: chred[a][r * cols + c] over the block's rpp rows ->
// pg / pb / dadd [b, c0..], in a fixed order by all threads: stage 1 sums 16-row chunks (one task per
// array x chunk x column), stage 2 the chunks in order.  (A loop of `cols` threads over every row was a
// serial chain of ~400 LDS reads that held its wave several microseconds behind the rest of the block.)
constexpr int kGnChunk = 16;
__device__ __forceinline__ void gn_column_sums(float4 (*chred)[kGnThreads], float4 (*tmp)[128], int cols, int rpp,
                                               int tid, float *pg, float *pb, float *dadd, size_t out0) {
    const int nch = (rpp + kGnChunk - 1) / kGnChunk;
    for (int task = tid; task < 3 * nch * cols; task += kGnThreads) {
        const int a = task / (nch * cols), rem = task - a * nch * cols, ch = rem / cols, c = rem - ch * cols;
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        const int r1 = min(rpp, (ch + 1) * kGnChunk);
        for (int r = ch * kGnChunk; r < r1; ++r) {
            const float4 v = chred[a][r * cols + c];
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        tmp[a][ch * cols + c] = s;
    }
    __syncthreads();
    if (tid < 3 * cols) {
        const int a = tid / cols, c = tid - a * cols;
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int ch = 0; ch < nch; ++ch) {
            const float4 v = tmp[a][ch * cols + c];
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        float *out = a == 0 ? pg : a == 1 ? pb : dadd;
        if (out) *reinterpret_cast<float4 *>(out + out0 + c * 4) = s;
    }
}

// Register-resident variants (T <= P * rows_per_pass): the group's values are loaded ONCE into
// registers -- one HBM read + one write per element instead of three / four streaming passes -- with
// the same per-thread summation order as the streaming kernels.
template <int P, typename TH, typename TY>
__global__ __launch_bounds__(kGnThreads) void gn_mish_fwd_reg_kernel(const TH *__restrict__ h, const float *__restrict__ gamma,
                                                                   const float *__restrict__ beta,
                                                                   const float *__restrict__ mask,
                                                                   const float *__restrict__ add, TY *__restrict__ y,
                                                                   float *__restrict__ mean_out,
                                                                   float *__restrict__ rstd_out, int T, int C, int G,
                                                                   float eps) {
    __shared__ float red[kGnThreads / 64];
    const int g = blockIdx.x, b = blockIdx.y;
    const int cg = C / G, cols = cg / 4, rpp = kGnThreads / cols;
    const int tid = threadIdx.x, col = tid % cols, r0 = tid / cols;
    const bool active = r0 < rpp;
    const int c0 = g * cg + col * 4;
    const TH *hb = h + (size_t)b * T * C + c0;
    const float n = (float)T * cg;
    float4 v[P];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int t = r0 + k * rpp;
        v[k] = (active && t < T) ? ld4(hb + (size_t)t * C) : make_float4(0.f, 0.f, 0.f, 0.f);
        s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
    }
    const float mean = block_sum<kGnThreads>(s, red) / n;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        if (!active || r0 + k * rpp >= T) continue;
        const float a = v[k].x - mean, bq = v[k].y - mean, cq = v[k].z - mean, d = v[k].w - mean;
        q += (a * a + bq * bq) + (cq * cq + d * d);
    }
    const float var = block_sum<kGnThreads>(q, red) / n;
    const float rstd = rsqrtf(var + eps);
    if (tid == 0) {
        mean_out[b * G + g] = mean;
        rstd_out[b * G + g] = rstd;
    }
    if (!active) return;
    const float4 ga = *reinterpret_cast<const float4 *>(gamma + c0);
    const float4 be = *reinterpret_cast<const float4 *>(beta + c0);
    float4 ad = make_float4(0.f, 0.f, 0.f, 0.f);
    if (add) ad = *reinterpret_cast<const float4 *>(add + (size_t)b * C + c0);
    TY *yb = y + (size_t)b * T * C + c0;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int t = r0 + k * rpp;
        if (t >= T) continue;
        const float m = mask ? mask[(size_t)b * T + t] : 1.f;
        float4 o;
        o.x = mish_f((v[k].x - mean) * rstd * ga.x + be.x) * m + ad.x;
        o.y = mish_f((v[k].y - mean) * rstd * ga.y + be.y) * m + ad.y;
        o.z = mish_f((v[k].z - mean) * rstd * ga.z + be.z) * m + ad.z;
        o.w = mish_f((v[k].w - mean) * rstd * ga.w + be.w) * m + ad.w;
        st4(yb + (size_t)t * C, o);
    }
}

// TD / TH / TO: storage of dy / h / dh (float or bf16 bits)
template <int P, typename TD, typename TH, typename TO>
__global__ __launch_bounds__(kGnThreads) void gn_mish_bwd_reg_kernel(
    const TD *__restrict__ dy, const TH *__restrict__ h, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ mask, const float *__restrict__ mean_in,
    const float *__restrict__ rstd_in, TO *__restrict__ dh, float *__restrict__ pg, float *__restrict__ pb,
    float *__restrict__ dadd, int T, int C, int G) {
    __shared__ float red[kGnThreads / 64];
    __shared__ float4 chred[3][kGnThreads];
    __shared__ float4 ctmp[3][128];
    const int g = blockIdx.x, b = blockIdx.y;
    const int cg = C / G, cols = cg / 4, rpp = kGnThreads / cols;
    const int tid = threadIdx.x, col = tid % cols, r0 = tid / cols;
    const bool active = r0 < rpp;
    const int c0 = g * cg + col * 4;
    const float mean = mean_in[b * G + g], rstd = rstd_in[b * G + g];
    const float4 ga = *reinterpret_cast<const float4 *>(gamma + c0);
    const float4 be = *reinterpret_cast<const float4 *>(beta + c0);
    const TH *hb = h + (size_t)b * T * C + c0;
    const TD *db_ = dy + (size_t)b * T * C + c0;
    const float n = (float)T * cg;
    float4 v[P], gu[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int t = r0 + k * rpp;
        const bool ok = active && t < T;
        v[k] = ok ? ld4(hb + (size_t)t * C) : make_float4(0.f, 0.f, 0.f, 0.f);
        gu[k] = ok ? ld4(db_ + (size_t)t * C) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float s1 = 0.f, s2 = 0.f;
    float4 ag = make_float4(0, 0, 0, 0), ab = make_float4(0, 0, 0, 0), ad = make_float4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int t = r0 + k * rpp;
        if (!active || t >= T) continue;
        const float m = mask ? mask[(size_t)b * T + t] : 1.f;
        float xh, d;
#define MTTS_GN_BWD_ACC(X, G_, GA, BE, AG, AB, AD) \
    xh = (X - mean) * rstd;                         \
    d = G_;                                          \
    G_ = d * m * mish_grad(xh * GA + BE);            \
    s1 += G_ * GA;                                   \
    s2 += G_ * GA * xh;                              \
    AG += G_ * xh;                                   \
    AB += G_;                                        \
    AD += d;
        MTTS_GN_BWD_ACC(v[k].x, gu[k].x, ga.x, be.x, ag.x, ab.x, ad.x)
        MTTS_GN_BWD_ACC(v[k].y, gu[k].y, ga.y, be.y, ag.y, ab.y, ad.y)
        MTTS_GN_BWD_ACC(v[k].z, gu[k].z, ga.z, be.z, ag.z, ab.z, ad.z)
        MTTS_GN_BWD_ACC(v[k].w, gu[k].w, ga.w, be.w, ag.w, ab.w, ad.w)
#undef MTTS_GN_BWD_ACC
    }
    const float m1 = block_sum<kGnThreads>(s1, red) / n;
    const float m2 = block_sum<kGnThreads>(s2, red) / n;
    chred[0][tid] = ag;
    chred[1][tid] = ab;
    chred[2][tid] = ad;
    __syncthreads();
    gn_column_sums(chred, ctmp, cols, rpp, tid, pg, pb, dadd, (size_t)b * C + g * cg);
    if (!active) return;
    TO *dhb = dh + (size_t)b * T * C + c0;
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int t = r0 + k * rpp;
        if (t >= T) continue;
        float4 o;
        o.x = rstd * (gu[k].x * ga.x - m1 - (v[k].x - mean) * rstd * m2);
        o.y = rstd * (gu[k].y * ga.y - m1 - (v[k].y - mean) * rstd * m2);
        o.z = rstd * (gu[k].z * ga.z - m1 - (v[k].z - mean) * rstd * m2);
        o.w = rstd * (gu[k].w * ga.w - m1 - (v[k].w - mean) * rstd * m2);
        st4(dhb + (size_t)t * C, o);
    }
}

// Backward.  Per element: u = xhat*gamma + beta, g_u = dy * mask * mish'(u), dxhat = g_u * gamma.
// dh = rstd * (dxhat - mean(dxhat) - xhat * mean(dxhat * xhat)) over the (b, g) group.
// Partial outputs per (b, c): pg[b,c] = sum_t g_u*xhat, pb[b,c] = sum_t g_u, dadd[b,c] = sum_t dy.
template <typename TD, typename TH, typename TO>
__global__ __launch_bounds__(kGnThreads) void gn_mish_bwd_kernel(
    const TD *__restrict__ dy, const TH *__restrict__ h, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ mask, const float *__restrict__ mean_in,
    const float *__restrict__ rstd_in, TO *__restrict__ dh, float *__restrict__ pg, float *__restrict__ pb,
    float *__restrict__ dadd, int T, int C, int G) {
    __shared__ float red[kGnThreads / 64];
    __shared__ float4 chred[3][kGnThreads];
    __shared__ float4 ctmp[3][128];
    const int g = blockIdx.x, b = blockIdx.y;
    const int cg = C / G;
    const int cols = cg / 4;
    const int rows_per_pass = kGnThreads / cols;
    const int tid = threadIdx.x;
    const int col = tid % cols, r0 = tid / cols;
    const bool active = r0 < rows_per_pass;
    const int c0 = g * cg + col * 4;
    const float mean = mean_in[b * G + g], rstd = rstd_in[b * G + g];
    const float4 ga = *reinterpret_cast<const float4 *>(gamma + c0);
    const float4 be = *reinterpret_cast<const float4 *>(beta + c0);
    const TH *hb = h + (size_t)b * T * C + c0;
    const TD *db_ = dy + (size_t)b * T * C + c0;
    const float n = (float)T * cg;

    float s1 = 0.f, s2 = 0.f;
    float4 ag = make_float4(0, 0, 0, 0), ab = make_float4(0, 0, 0, 0), ad = make_float4(0, 0, 0, 0);
    if (active)
        for (int t = r0; t < T; t += rows_per_pass) {
            const float4 v = ld4(hb + (size_t)t * C);
            const float4 d = ld4(db_ + (size_t)t * C);
            const float m = mask ? mask[(size_t)b * T + t] : 1.f;
            float xh, gu;
#define MTTS_GN_BWD_ACC(X, D, GA, BE, AG, AB, AD)          \
    xh = (X - mean) * rstd;                                 \
    gu = D * m * mish_grad(xh * GA + BE);                   \
    s1 += gu * GA;                                          \
    s2 += gu * GA * xh;                                     \
    AG += gu * xh;                                          \
    AB += gu;                                               \
    AD += D;
            MTTS_GN_BWD_ACC(v.x, d.x, ga.x, be.x, ag.x, ab.x, ad.x)
            MTTS_GN_BWD_ACC(v.y, d.y, ga.y, be.y, ag.y, ab.y, ad.y)
            MTTS_GN_BWD_ACC(v.z, d.z, ga.z, be.z, ag.z, ab.z, ad.z)
            MTTS_GN_BWD_ACC(v.w, d.w, ga.w, be.w, ag.w, ab.w, ad.w)
#undef MTTS_GN_BWD_ACC
        }
    const float m1 = block_sum<kGnThreads>(s1, red) / n;
    const float m2 = block_sum<kGnThreads>(s2, red) / n;
    // per-channel partials: reduce the rows_per_pass threads that share a column, fixed order
    chred[0][tid] = ag;
    chred[1][tid] = ab;
    chred[2][tid] = ad;
    __syncthreads();
    gn_column_sums(chred, ctmp, cols, rows_per_pass, tid, pg, pb, dadd, (size_t)b * C + g * cg);
    if (!active) return;
    TO *dhb = dh + (size_t)b * T * C + c0;
    for (int t = r0; t < T; t += rows_per_pass) {
        const float4 v = ld4(hb + (size_t)t * C);
        const float4 d = ld4(db_ + (size_t)t * C);
        const float m = mask ? mask[(size_t)b * T + t] : 1.f;
        float4 o;
        float xh, gu;
#define MTTS_GN_BWD_OUT(X, D, GA, BE, O)                     \
    xh = (X - mean) * rstd;                                   \
    gu = D * m * mish_grad(xh * GA + BE);                     \
    O = rstd * (gu * GA - m1 - xh * m2);
        MTTS_GN_BWD_OUT(v.x, d.x, ga.x, be.x, o.x)
        MTTS_GN_BWD_OUT(v.y, d.y, ga.y, be.y, o.y)
        MTTS_GN_BWD_OUT(v.z, d.z, ga.z, be.z, o.z)
        MTTS_GN_BWD_OUT(v.w, d.w, ga.w, be.w, o.w)
#undef MTTS_GN_BWD_OUT
        st4(dhb + (size_t)t * C, o);
    }
}

// gamma/beta gradients = fixed-order sums of the [R][C] per-block partials (reduce.hip: now, or
// queued for the step's batched launch)
int submit_param_sums(const float *pa, float *outa, const float *pb, float *outb, int R, int C, hipStream_t st) {
    mtts_reduce_job jobs[2] = {};
    int n = 0;
    for (int w = 0; w < 2; ++w) {
        float *out = w ? outb : outa;
        if (!out) continue;
        jobs[n].part = w ? pb : pa;
        jobs[n].out = out;
        jobs[n].stride = C;
        jobs[n].n = C;
        jobs[n].splits = R;
        ++n;
    }
    return n ? mtts::submit_reductions(jobs, n, st) : MTTS_OK;
}

// ------------------------------------------------------------------------------ LayerNorm
// Each wave normalises R consecutive rows, all their loads (and the affine weights') issued before the
// first reduction; lane handles float4 chunks lane*4 + 256*i, NI chunks (C <= 256 * NI).  One row per
// wave kept ~1 KB in flight per wave -- well under what a CU needs to stream at its HBM share.
template <bool Y16, int NI, int R>  // Y16: y written as bf16 (MTTS_NORM_F_Y_BF16)
__global__ __launch_bounds__(kThreads) void layernorm_fwd_kernel(const float *__restrict__ x, const float *__restrict__ w,
                                                                 const float *__restrict__ bia, float *__restrict__ y,
                                                                 float *__restrict__ mean_out, float *__restrict__ rstd_out,
                                                                 int M, int C, float eps, int act, float p,
                                                                 const uint32_t *__restrict__ seed) {
    const int row0 = (blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6)) * R;
    const int lane = threadIdx.x & 63;
    if (row0 >= M) return;
    float4 v[R][NI], ww[NI], bb[NI];
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const float *xr = x + (size_t)(row0 + q) * C;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int c = lane * 4 + 256 * i;
            v[q][i] = row0 + q < M && c < C ? *reinterpret_cast<const float4 *>(xr + c) : make_float4(0, 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int c = lane * 4 + 256 * i;
        ww[i] = c < C ? *reinterpret_cast<const float4 *>(w + c) : make_float4(0, 0, 0, 0);
        bb[i] = c < C ? *reinterpret_cast<const float4 *>(bia + c) : make_float4(0, 0, 0, 0);
    }
    uint32_t sd0 = 0, sd1 = 0;  // dropout seed words
    if (p > 0.f) {
        sd0 = seed[0];
        sd1 = seed[1];
    }
    const float inv_keep = mtts::dropout_scale(p);
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int row = row0 + q;
        if (row >= M) break;  // wave-uniform
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i) s += (v[q][i].x + v[q][i].y) + (v[q][i].z + v[q][i].w);
        const float mean = wave_sum(s) / C;
        float sq = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int c = lane * 4 + 256 * i;
            if (c < C) {
                const float a = v[q][i].x - mean, b = v[q][i].y - mean, cc = v[q][i].z - mean, d = v[q][i].w - mean;
                sq += (a * a + b * b) + (cc * cc + d * d);
            }
        }
        const float rstd = rsqrtf(wave_sum(sq) / C + eps);
        if (lane == 0) {
            mean_out[row] = mean;
            rstd_out[row] = rstd;
        }
        float *yr = y + (size_t)row * C;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int c = lane * 4 + 256 * i;
            if (c < C) {
                float o[4] = {(v[q][i].x - mean) * rstd * ww[i].x + bb[i].x, (v[q][i].y - mean) * rstd * ww[i].y + bb[i].y,
                              (v[q][i].z - mean) * rstd * ww[i].z + bb[i].z, (v[q][i].w - mean) * rstd * ww[i].w + bb[i].w};
                if (act == MTTS_ACT_RELU || p > 0.f) {  // fused tail: ReLU then dropout (ConvReluNorm order)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (act == MTTS_ACT_RELU) o[j] = fmaxf(o[j], 0.f);
                        if (p > 0.f) o[j] = mtts::dropout_keep(sd0, sd1, (uint32_t)row, (uint32_t)(c + j), p) ? o[j] * inv_keep : 0.f;
                    }
                }
                if constexpr (Y16) {
                    typedef float f2 __attribute__((ext_vector_type(2)));
                    typedef __bf16 h2 __attribute__((ext_vector_type(2)));
                    const uint32_t lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){o[0], o[1]}, h2));
                    const uint32_t hi = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){o[2], o[3]}, h2));
                    *reinterpret_cast<uint2 *>(reinterpret_cast<uint16_t *>(y) + (size_t)row * C + c) = make_uint2(lo, hi);
                } else {
                    *reinterpret_cast<float4 *>(yr + c) = make_float4(o[0], o[1], o[2], o[3]);
                }
            }
        }
    }
}

// backward: each wave takes R consecutive rows at once (all their loads issued before the first
// reduction), the block 4 * R rows per pass, rows_per_block a multiple of that sized for ~768 blocks
// (at most 128 rows).  One row per wave at a time left the decoder's 19200-row LayerNorms (40 rows per
// block, 10 dependent load -> reduce -> store rounds per wave) latency-bound at 12-22 us.
// NI: float4 chunks per lane (1: C <= 256, 4: C <= 1024).
inline int ln_bwd_rows_in_flight(int C) { return C <= 256 ? 4 : 1; }
inline int ln_rows_per_block(int M, int C) {
    const int q = 4 * ln_bwd_rows_in_flight(C);  // rows per block pass
    int r = (M + 767) / 768;
    r = (r + q - 1) / q * q;
    return r < q ? q : (r > 128 ? 128 : r);
}

template <int NI, int R>
__global__ __launch_bounds__(kThreads) void layernorm_bwd_kernel(const float *__restrict__ dy, const float *__restrict__ x,
                                                                 const float *__restrict__ w, const float *__restrict__ bia,
                                                                 const float *__restrict__ mean_in,
                                                                 const float *__restrict__ rstd_in, float *__restrict__ dx,
                                                                 float *__restrict__ pw, float *__restrict__ pb, int M,
                                                                 int C, int act, float p, const uint32_t *__restrict__ seed,
                                                                 int rows_per_block, const float *__restrict__ dres) {
    __shared__ float4 red[2][kThreads / 64][64 * NI];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float4 aw[NI], ab[NI], ww[NI], bb[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int c = lane * 4 + 256 * i;
        aw[i] = ab[i] = make_float4(0, 0, 0, 0);
        ww[i] = c < C ? *reinterpret_cast<const float4 *>(w + c) : make_float4(0, 0, 0, 0);
        bb[i] = (c < C && act == MTTS_ACT_RELU) ? *reinterpret_cast<const float4 *>(bia + c) : make_float4(0, 0, 0, 0);
    }
    const bool tail = act == MTTS_ACT_RELU || p > 0.f;
    uint32_t sd0 = 0, sd1 = 0;  // dropout seed words
    if (p > 0.f) {
        sd0 = seed[0];
        sd1 = seed[1];
    }
    const float inv_keep = mtts::dropout_scale(p);
    const int rbeg = blockIdx.x * rows_per_block;
    const int rend = min(M, rbeg + rows_per_block);
    for (int r0 = rbeg + wv * R; r0 < rend; r0 += (kThreads / 64) * R) {
        float4 xv[R][NI], dv[R][NI], rv[R][NI];
        float mean[R], rstd[R];
#pragma unroll
        for (int q = 0; q < R; ++q) {  // every load of the R rows first
            const int row = r0 + q;
            const bool ok = row < rend;
            mean[q] = ok ? mean_in[row] : 0.f;
            rstd[q] = ok ? rstd_in[row] : 0.f;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int c = lane * 4 + 256 * i;
                const bool in = ok && c < C;
                xv[q][i] = in ? *reinterpret_cast<const float4 *>(x + (size_t)row * C + c) : make_float4(0, 0, 0, 0);
                dv[q][i] = in ? *reinterpret_cast<const float4 *>(dy + (size_t)row * C + c) : make_float4(0, 0, 0, 0);
                rv[q][i] = in && dres ? *reinterpret_cast<const float4 *>(dres + (size_t)row * C + c) : make_float4(0, 0, 0, 0);
            }
        }
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int row = r0 + q;
            if (row >= rend) break;  // wave-uniform
            float4 xh[NI], g[NI];
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int c = lane * 4 + 256 * i;
                if (c < C) {
                    const float4 xq = xv[q][i];
                    float4 d = dv[q][i];
                    xh[i] = make_float4((xq.x - mean[q]) * rstd[q], (xq.y - mean[q]) * rstd[q], (xq.z - mean[q]) * rstd[q],
                                        (xq.w - mean[q]) * rstd[q]);
                    if (tail) {  // through the fused tail: regenerate the dropout mask, ReLU gate from the LN output
                        float d4[4] = {d.x, d.y, d.z, d.w};
                        const float xs[4] = {xh[i].x, xh[i].y, xh[i].z, xh[i].w};
                        const float w4[4] = {ww[i].x, ww[i].y, ww[i].z, ww[i].w};
                        const float b4[4] = {bb[i].x, bb[i].y, bb[i].z, bb[i].w};
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            if (p > 0.f)
                                d4[j] = mtts::dropout_keep(sd0, sd1, (uint32_t)row, (uint32_t)(c + j), p) ? d4[j] * inv_keep : 0.f;
                            if (act == MTTS_ACT_RELU && xs[j] * w4[j] + b4[j] <= 0.f) d4[j] = 0.f;
                        }
                        d = make_float4(d4[0], d4[1], d4[2], d4[3]);
                    }
                    g[i] = make_float4(d.x * ww[i].x, d.y * ww[i].y, d.z * ww[i].z, d.w * ww[i].w);
                    s1 += (g[i].x + g[i].y) + (g[i].z + g[i].w);
                    s2 += (g[i].x * xh[i].x + g[i].y * xh[i].y) + (g[i].z * xh[i].z + g[i].w * xh[i].w);
                    aw[i].x += d.x * xh[i].x; aw[i].y += d.y * xh[i].y; aw[i].z += d.z * xh[i].z; aw[i].w += d.w * xh[i].w;
                    ab[i].x += d.x; ab[i].y += d.y; ab[i].z += d.z; ab[i].w += d.w;
                }
            }
            const float m1 = wave_sum(s1) / C, m2 = wave_sum(s2) / C;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int c = lane * 4 + 256 * i;
                if (c < C) {
                    float4 o;
                    o.x = rstd[q] * (g[i].x - m1 - xh[i].x * m2);
                    o.y = rstd[q] * (g[i].y - m1 - xh[i].y * m2);
                    o.z = rstd[q] * (g[i].z - m1 - xh[i].z * m2);
                    o.w = rstd[q] * (g[i].w - m1 - xh[i].w * m2);
                    if (dres) {  // + the residual branch's gradient (pre-LN block: x feeds the LN and the residual)
                        o.x += rv[q][i].x; o.y += rv[q][i].y; o.z += rv[q][i].z; o.w += rv[q][i].w;
                    }
                    *reinterpret_cast<float4 *>(dx + (size_t)row * C + c) = o;
                }
            }
        }
    }
    // reduce the 4 waves' partials (fixed order) -> one [C] partial per block
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int c4 = lane + 64 * i;  // float4 index
        if (c4 * 4 < C) {
            red[0][wv][c4] = aw[i];
            red[1][wv][c4] = ab[i];
        }
    }
    __syncthreads();
    for (int c4 = threadIdx.x; c4 * 4 < C; c4 += kThreads) {
        float4 sw = make_float4(0, 0, 0, 0), sb = sw;
        for (int q = 0; q < kThreads / 64; ++q) {
            const float4 a = red[0][q][c4], bb = red[1][q][c4];
            sw.x += a.x; sw.y += a.y; sw.z += a.z; sw.w += a.w;
            sb.x += bb.x; sb.y += bb.y; sb.z += bb.z; sb.w += bb.w;
        }
        *reinterpret_cast<float4 *>(pw + (size_t)blockIdx.x * C + c4 * 4) = sw;
        *reinterpret_cast<float4 *>(pb + (size_t)blockIdx.x * C + c4 * 4) = sb;
    }
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

template <typename TH, typename TY>
static void gn_fwd_launch(const void *h, const float *gamma, const float *beta, const float *mask, const float *add,
                          void *y, float *mean, float *rstd, int B, int T, int C, int G, float eps, hipStream_t st) {
    const TH *hh = static_cast<const TH *>(h);
    TY *yy = static_cast<TY *>(y);
    const int passes = (T + kGnThreads / (C / G / 4) - 1) / (kGnThreads / (C / G / 4));
    if (passes <= 4)
        hipLaunchKernelGGL((gn_mish_fwd_reg_kernel<4, TH, TY>), dim3(G, B), dim3(kGnThreads), 0, st, hh, gamma, beta,
                           mask, add, yy, mean, rstd, T, C, G, eps);
    else if (passes <= 8)
        hipLaunchKernelGGL((gn_mish_fwd_reg_kernel<8, TH, TY>), dim3(G, B), dim3(kGnThreads), 0, st, hh, gamma, beta,
                           mask, add, yy, mean, rstd, T, C, G, eps);
    else
        hipLaunchKernelGGL((gn_mish_fwd_kernel<TH, TY>), dim3(G, B), dim3(kGnThreads), 0, st, hh, gamma, beta, mask, add,
                           yy, mean, rstd, T, C, G, eps);
}

extern "C" int mtts_gn_mish_fwd_ex(const void *h, const float *gamma, const float *beta, const float *mask,
                                   const float *add, void *y, float *mean, float *rstd, int32_t B, int32_t T,
                                   int32_t C, int32_t G, float eps, int32_t flags, void *hip_stream) {
    MTTS_CHECK_ARG(h && gamma && beta && y && mean && rstd, "gn_mish_fwd: null pointer");
    MTTS_CHECK_ARG(B >= 0 && T >= 1 && G >= 1 && C % G == 0 && (C / G) % 4 == 0 && C / G <= 4 * kGnThreads,
                   "gn_mish_fwd: need C % G == 0 and (C/G) % 4 == 0");
    MTTS_CHECK_ARG(!(flags & ~(MTTS_NORM_F_X_BF16 | MTTS_NORM_F_Y_BF16)), "gn_mish_fwd: unknown flag");
    MTTS_CHECK_ARG(aligned16(h) && aligned16(y) && aligned16(gamma) && aligned16(beta) && (!add || aligned16(add)),
                   "gn_mish_fwd: tensors must be 16-byte aligned");
    if (B == 0) return MTTS_OK;
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    const bool x16 = flags & MTTS_NORM_F_X_BF16, y16 = flags & MTTS_NORM_F_Y_BF16;
    if (x16 && y16) gn_fwd_launch<uint16_t, uint16_t>(h, gamma, beta, mask, add, y, mean, rstd, B, T, C, G, eps, st);
    else if (x16) gn_fwd_launch<uint16_t, float>(h, gamma, beta, mask, add, y, mean, rstd, B, T, C, G, eps, st);
    else if (y16) gn_fwd_launch<float, uint16_t>(h, gamma, beta, mask, add, y, mean, rstd, B, T, C, G, eps, st);
    else gn_fwd_launch<float, float>(h, gamma, beta, mask, add, y, mean, rstd, B, T, C, G, eps, st);
    return mtts::check_launch("gn_mish_fwd_kernel");
}

extern "C" int mtts_gn_mish_fwd(const float *h, const float *gamma, const float *beta, const float *mask,
                                const float *add, float *y, float *mean, float *rstd, int32_t B, int32_t T,
                                int32_t C, int32_t G, float eps, void *hip_stream) {
    return mtts_gn_mish_fwd_ex(h, gamma, beta, mask, add, y, mean, rstd, B, T, C, G, eps, 0, hip_stream);
}

extern "C" size_t mtts_gn_mish_bwd_workspace_size(int32_t B, int32_t C) {
    return (size_t)2 * (B > 0 ? B : 0) * (C > 0 ? C : 0) * sizeof(float);
}

template <typename TD, typename TH, typename TO>
static void gn_bwd_launch(const void *dy, const void *h, const float *gamma, const float *beta, const float *mask,
                          const float *mean, const float *rstd, void *dh, float *pg, float *pb, float *dadd, int B,
                          int T, int C, int G, hipStream_t st) {
    const TD *d = static_cast<const TD *>(dy);
    const TH *hh = static_cast<const TH *>(h);
    TO *o = static_cast<TO *>(dh);
    const int passes = (T + kGnThreads / (C / G / 4) - 1) / (kGnThreads / (C / G / 4));
    if (passes <= 4)
        hipLaunchKernelGGL((gn_mish_bwd_reg_kernel<4, TD, TH, TO>), dim3(G, B), dim3(kGnThreads), 0, st, d, hh, gamma,
                           beta, mask, mean, rstd, o, pg, pb, dadd, T, C, G);
    else if (passes <= 6)  // (8 spills at 1024 threads)
        hipLaunchKernelGGL((gn_mish_bwd_reg_kernel<6, TD, TH, TO>), dim3(G, B), dim3(kGnThreads), 0, st, d, hh, gamma,
                           beta, mask, mean, rstd, o, pg, pb, dadd, T, C, G);
    else
        hipLaunchKernelGGL((gn_mish_bwd_kernel<TD, TH, TO>), dim3(G, B), dim3(kGnThreads), 0, st, d, hh, gamma, beta,
                           mask, mean, rstd, o, pg, pb, dadd, T, C, G);
}

extern "C" int mtts_gn_mish_bwd_ex(const void *dy, const void *h, const float *gamma, const float *beta,
                                   const float *mask, const float *mean, const float *rstd, void *dh, float *dgamma,
                                   float *dbeta, float *dadd, int32_t B, int32_t T, int32_t C, int32_t G,
                                   int32_t flags, void *workspace, size_t workspace_bytes, void *hip_stream) {
    MTTS_CHECK_ARG(dy && h && gamma && beta && mean && rstd && dh, "gn_mish_bwd: null pointer");
    MTTS_CHECK_ARG(B >= 0 && T >= 1 && G >= 1 && C % G == 0 && (C / G) % 4 == 0 && C / G <= 256,
                   "gn_mish_bwd: need C % G == 0, (C/G) % 4 == 0 and C/G <= 256");
    MTTS_CHECK_ARG(aligned16(dy) && aligned16(h) && aligned16(dh) && (!dadd || aligned16(dadd)),
                   "gn_mish_bwd: tensors must be 16-byte aligned");
    const int known = MTTS_NORM_F_X_BF16 | MTTS_NORM_F_Y_BF16 | MTTS_NORM_F_DY_BF16;
    MTTS_CHECK_ARG(!(flags & ~known), "gn_mish_bwd: unknown flag");
    if (B == 0) return MTTS_OK;
    if (!workspace || workspace_bytes < mtts_gn_mish_bwd_workspace_size(B, C))
        return mtts::fail(MTTS_ERR_WORKSPACE, "gn_mish_bwd: workspace too small");
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    float *pg = static_cast<float *>(workspace);
    float *pb = pg + (size_t)B * C;
    // the storage combinations the decoder runs: all fp32 (32-true); bf16 h and dh with fp32 or bf16 dy
    switch (flags) {
        case 0:
            gn_bwd_launch<float, float, float>(dy, h, gamma, beta, mask, mean, rstd, dh, pg, pb, dadd, B, T, C, G, st);
            break;
        case MTTS_NORM_F_X_BF16 | MTTS_NORM_F_Y_BF16:
            gn_bwd_launch<float, uint16_t, uint16_t>(dy, h, gamma, beta, mask, mean, rstd, dh, pg, pb, dadd, B, T, C, G, st);
            break;
        case MTTS_NORM_F_X_BF16 | MTTS_NORM_F_Y_BF16 | MTTS_NORM_F_DY_BF16:
            gn_bwd_launch<uint16_t, uint16_t, uint16_t>(dy, h, gamma, beta, mask, mean, rstd, dh, pg, pb, dadd, B, T, C,
                                                        G, st);
            break;
        default:
            return mtts::fail(MTTS_ERR_UNSUPPORTED, "gn_mish_bwd: unsupported storage combination");
    }
    int rc = mtts::check_launch("gn_mish_bwd_kernel");
    if (rc) return rc;
    return submit_param_sums(pg, dgamma, pb, dbeta, B, C, st);
}

extern "C" int mtts_gn_mish_bwd(const float *dy, const float *h, const float *gamma, const float *beta,
                                const float *mask, const float *mean, const float *rstd, float *dh, float *dgamma,
                                float *dbeta, float *dadd, int32_t B, int32_t T, int32_t C, int32_t G,
                                void *workspace, size_t workspace_bytes, void *hip_stream) {
    return mtts_gn_mish_bwd_ex(dy, h, gamma, beta, mask, mean, rstd, dh, dgamma, dbeta, dadd, B, T, C, G, 0, workspace,
                               workspace_bytes, hip_stream);
}

extern "C" int mtts_layernorm_fwd(const float *x, const float *w, const float *b, float *y, float *mean,
                                  float *rstd, int32_t M, int32_t C, float eps, int32_t act, float dropout_p,
                                  const uint32_t *seed, void *hip_stream) {
    MTTS_CHECK_ARG(x && w && b && y && mean && rstd, "layernorm_fwd: null pointer");
    const bool y16 = act & MTTS_NORM_F_Y_BF16;
    act &= ~MTTS_NORM_F_Y_BF16;
    MTTS_CHECK_ARG(act == MTTS_ACT_NONE || act == MTTS_ACT_RELU, "layernorm_fwd: act must be NONE or RELU");
    MTTS_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || seed), "layernorm_fwd: bad dropout");
    MTTS_CHECK_ARG(M >= 0 && C >= 4 && C % 4 == 0 && C <= 1024, "layernorm_fwd: need C % 4 == 0, C <= 1024");
    MTTS_CHECK_ARG(aligned16(x) && aligned16(y) && aligned16(w) && aligned16(b), "layernorm_fwd: 16-byte alignment");
    if (M == 0) return MTTS_OK;
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    // 4 rows per wave (C <= 256) once the grid still has >= 2 blocks per CU; else one
    const int R = C <= 256 && M >= 4 * 4 * 512 ? 4 : 1;
    const dim3 grid((M + 4 * R - 1) / (4 * R));
#define MTTS_LN_FWD(Y, NI, RR)                                                                                          \
    hipLaunchKernelGGL((layernorm_fwd_kernel<Y, NI, RR>), grid, dim3(kThreads), 0, st, x, w, b, y, mean, rstd, M, C, eps, \
                       act, dropout_p, seed)
    if (C > 256) {
        if (y16) MTTS_LN_FWD(true, 4, 1);
        else MTTS_LN_FWD(false, 4, 1);
    } else if (R == 4) {
        if (y16) MTTS_LN_FWD(true, 1, 4);
        else MTTS_LN_FWD(false, 1, 4);
    } else {
        if (y16) MTTS_LN_FWD(true, 1, 1);
        else MTTS_LN_FWD(false, 1, 1);
    }
#undef MTTS_LN_FWD
    return mtts::check_launch("layernorm_fwd_kernel");
}

extern "C" size_t mtts_layernorm_bwd_workspace_size(int32_t M, int32_t C) {
    if (M <= 0 || C <= 0) return 0;
    const int rpb = ln_rows_per_block(M, C);
    return (size_t)2 * ((M + rpb - 1) / rpb) * C * sizeof(float);
}

static int layernorm_bwd_impl(const float *dy, const float *x, const float *w, const float *b, const float *mean,
                              const float *rstd, const float *dres, float *dx, float *dw, float *db, int32_t M,
                              int32_t C, int32_t act, float dropout_p, const uint32_t *seed, void *workspace,
                              size_t workspace_bytes, void *hip_stream) {
    MTTS_CHECK_ARG(dy && x && w && mean && rstd && dx, "layernorm_bwd: null pointer");
    MTTS_CHECK_ARG(!dres || aligned16(dres), "layernorm_bwd: dres must be 16-byte aligned");
    MTTS_CHECK_ARG(act == MTTS_ACT_NONE || (act == MTTS_ACT_RELU && b), "layernorm_bwd: act RELU needs b");
    MTTS_CHECK_ARG(dropout_p >= 0.f && dropout_p < 1.f && (dropout_p == 0.f || seed), "layernorm_bwd: bad dropout");
    MTTS_CHECK_ARG(M >= 0 && C >= 4 && C % 4 == 0 && C <= 1024, "layernorm_bwd: need C % 4 == 0, C <= 1024");
    MTTS_CHECK_ARG(aligned16(dy) && aligned16(x) && aligned16(dx) && aligned16(w), "layernorm_bwd: 16-byte alignment");
    if (M == 0) return MTTS_OK;
    if (!workspace || workspace_bytes < mtts_layernorm_bwd_workspace_size(M, C))
        return mtts::fail(MTTS_ERR_WORKSPACE, "layernorm_bwd: workspace too small");
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    const int rpb = ln_rows_per_block(M, C);
    const int nblk = (M + rpb - 1) / rpb;
    float *pw = static_cast<float *>(workspace);
    float *pb = pw + (size_t)nblk * C;
    if (C <= 256)
        hipLaunchKernelGGL((layernorm_bwd_kernel<1, 4>), dim3(nblk), dim3(kThreads), 0, st, dy, x, w, b, mean, rstd, dx,
                           pw, pb, M, C, act, dropout_p, seed, rpb, dres);
    else
        hipLaunchKernelGGL((layernorm_bwd_kernel<4, 1>), dim3(nblk), dim3(kThreads), 0, st, dy, x, w, b, mean, rstd, dx,
                           pw, pb, M, C, act, dropout_p, seed, rpb, dres);
    int rc = mtts::check_launch("layernorm_bwd_kernel");
    if (rc) return rc;
    return submit_param_sums(pw, dw, pb, db, nblk, C, st);
}

extern "C" int mtts_layernorm_bwd(const float *dy, const float *x, const float *w, const float *b, const float *mean,
                                  const float *rstd, float *dx, float *dw, float *db, int32_t M, int32_t C,
                                  int32_t act, float dropout_p, const uint32_t *seed, void *workspace,
                                  size_t workspace_bytes, void *hip_stream) {
    return layernorm_bwd_impl(dy, x, w, b, mean, rstd, nullptr, dx, dw, db, M, C, act, dropout_p, seed, workspace,
                              workspace_bytes, hip_stream);
}

extern "C" int mtts_layernorm_bwd_res(const float *dy, const float *x, const float *w, const float *b,
                                      const float *mean, const float *rstd, const float *dres, float *dx, float *dw,
                                      float *db, int32_t M, int32_t C, void *workspace, size_t workspace_bytes,
                                      void *hip_stream) {
    return layernorm_bwd_impl(dy, x, w, b, mean, rstd, dres, dx, dw, db, M, C, MTTS_ACT_NONE, 0.f, nullptr, workspace,
                              workspace_bytes, hip_stream);
}
