// Shared epilogue of the conv/linear implicit GEMMs (conv_gemm.hip, conv_gemm_glds.hip).
//
// One wave holds TM x TN accumulators of v_mfma_f32_32x32x16 / 32x32x2 layout: register v of lane
// (lr = lane & 31, lh = lane >> 5) is C[row (v & 3) + 8 (v >> 2) + 4 lh][col lr] of its 32x32 tile.
// Per element: + bias[n] -> (store pre-activation) -> act -> dropout -> + residual -> * c_scale ->
// store at row b*To_full + u*out_stride + out_off of C.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mtts_common.h"
#include "mtts_decoder.h"

namespace mtts {

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
// epilogues VALU-heavy.  The fp32 parity mode keeps erff.  Round 5: t = 1 / (1 + p|z|) by v_rcp_f32 (1 ulp)
// instead of __frcp_rn, which hipcc expands to the IEEE division sequence (div_scale, rcp, two Newton steps,
// div_fmas, div_fixup: 10 of the ~24 VALU instructions of a GELU); the erf error bound is unchanged at fp32
// resolution.
__device__ __forceinline__ float erf_as_pdf(float z, float &ez2) {  // erf(z), ez2 = exp(-z^2)
    const float a = fabsf(z);
    const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * a);
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

typedef float f32x16 __attribute__((ext_vector_type(16)));

// b = m / d, u = m % d for 0 <= m < 2^24 with a precomputed 1/d (float estimate + one correction)
__device__ __forceinline__ void divmod_fast(int m, int d, float inv_d, int &q, int &r) {
    q = (int)((float)m * inv_d);
    r = m - q * d;
    if (r < 0) { --q; r += d; } else if (r >= d) { ++q; r -= d; }
}

// XCD-contiguous relabelling of a 1-D grid: the dispatcher deals consecutive block ids round-robin
// over the 8 XCDs, so block id b becomes the (b % 8)-th contiguous run of tiles (bijective for any
// grid size); with tiles numbered N-fastest the column blocks of one row panel share an XCD's L2.
__device__ __forceinline__ int xcd_relabel(int orig, int nwg) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

template <int TM, int TN>
__device__ __forceinline__ void gemm_epilogue(const mtts_conv_gemm_args &p, f32x16 (&acc)[TM][TN], int row0,
                                              int col0, int lr, int lh) {
    const int M = p.nb * p.To;
    const float inv_to = 1.0f / (float)p.To;
    uint32_t s0 = 0, s1 = 0;
    if (p.dropout_p > 0.f) {
        s0 = p.seed[0];
        s1 = p.seed[1];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        int crows[16];  // output row of each accumulator register (-1: past M)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int m = row0 + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * lh;
            int b, u;
            divmod_fast(m, p.To, inv_to, b, u);
            crows[v] = m < M ? b * p.To_full + u * p.out_stride + p.out_off : -1;
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = col0 + j * 32 + lr;
            if (n >= p.N) continue;
            const float bn = p.bias ? p.bias[n] : 0.f;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                if (crows[v] < 0) continue;
                const size_t crow = (size_t)crows[v];
                float val = acc[i][j][v] + bn;
                const bool pre16 = p.flags & MTTS_GEMM_F_PRE_BF16;
                if (p.C_pre) {
                    if (pre16) reinterpret_cast<__bf16 *>(p.C_pre)[crow * p.ldc + n] = (__bf16)val;
                    else p.C_pre[crow * p.ldc + n] = val;
                }
                if (p.act) {
                    float a = 0.f;
                    if (p.aux) a = pre16 ? (float)reinterpret_cast<const __bf16 *>(p.aux)[crow * p.ldaux + n]
                                         : p.aux[crow * p.ldaux + n];
                    val = epi_act(p.act, val, &a, p.flags & MTTS_GEMM_F_FAST_ACT);
                }
                if (p.dropout_p > 0.f)
                    val = dropout_keep(s0, s1, (uint32_t)crow, (uint32_t)n, p.dropout_p)
                              ? val * (1.0f / (1.0f - p.dropout_p))
                              : 0.f;
                if (p.residual) val += p.residual[crow * p.ldr + n];
                if (p.c_scale) val *= p.c_scale[crow];
                if (p.flags & MTTS_GEMM_F_C_BF16)
                    reinterpret_cast<__bf16 *>(p.C)[crow * p.ldc + n] = (__bf16)val;
                else
                    p.C[crow * p.ldc + n] = val;
            }
        }
    }
}

// Everything after the bias for 4 consecutive columns n..n+3 of output row crow (float4 I/O).
__device__ __forceinline__ void epilogue_row4(const mtts_conv_gemm_args &p, int crow, int n, float (&e)[4],
                                              uint32_t s0, uint32_t s1, float keep_scale) {
    typedef float f32x2_ __attribute__((ext_vector_type(2)));
    typedef __bf16 bf16x2_ __attribute__((ext_vector_type(2)));
    const size_t off = (size_t)crow * p.ldc + n;
    const bool pre16 = p.flags & MTTS_GEMM_F_PRE_BF16;
    if (p.C_pre) {
        if (pre16) {
            const uint32_t lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_){e[0], e[1]}, bf16x2_));
            const uint32_t hi = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_){e[2], e[3]}, bf16x2_));
            *reinterpret_cast<uint2 *>(reinterpret_cast<uint16_t *>(p.C_pre) + off) = make_uint2(lo, hi);
        } else {
            *reinterpret_cast<float4 *>(p.C_pre + off) = make_float4(e[0], e[1], e[2], e[3]);
        }
    }
    if (p.act) {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        if (p.act == MTTS_ACT_DGELU || p.act == MTTS_ACT_DRELU) {
            const size_t ao = (size_t)crow * p.ldaux + n;
            if (pre16) {  // bf16 -> fp32 is exact: the bits move to the high half
                const uint2 h = *reinterpret_cast<const uint2 *>(reinterpret_cast<const uint16_t *>(p.aux) + ao);
                a = make_float4(__uint_as_float(h.x << 16), __uint_as_float(h.x & 0xffff0000u),
                                __uint_as_float(h.y << 16), __uint_as_float(h.y & 0xffff0000u));
            } else {
                a = *reinterpret_cast<const float4 *>(p.aux + ao);
            }
        }
        const float av[4] = {a.x, a.y, a.z, a.w};
        const bool fast = p.flags & MTTS_GEMM_F_FAST_ACT;
#pragma unroll
        for (int q = 0; q < 4; ++q) e[q] = epi_act(p.act, e[q], &av[q], fast);
    }
    if (p.dropout_p > 0.f) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            e[q] = dropout_keep(s0, s1, (uint32_t)crow, (uint32_t)(n + q), p.dropout_p) ? e[q] * keep_scale : 0.f;
    }
    if (p.residual) {
        const float4 r = *reinterpret_cast<const float4 *>(p.residual + (size_t)crow * p.ldr + n);
        e[0] += r.x; e[1] += r.y; e[2] += r.z; e[3] += r.w;
    }
    if (p.c_scale) {
        const float cs = p.c_scale[crow];
#pragma unroll
        for (int q = 0; q < 4; ++q) e[q] *= cs;
    }
    if (p.flags & MTTS_GEMM_F_C_BF16) {
        const uint32_t lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_){e[0], e[1]}, bf16x2_));
        const uint32_t hi = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_){e[2], e[3]}, bf16x2_));
        *reinterpret_cast<uint2 *>(reinterpret_cast<uint16_t *>(p.C) + off) = make_uint2(lo, hi);
    } else {
        *reinterpret_cast<float4 *>(p.C + off) = make_float4(e[0], e[1], e[2], e[3]);
    }
}

// Split-K partial store: the raw accumulators of a wave's tiles into part[M][N] (row = GEMM row),
// through the same per-wave LDS image as gemm_epilogue_vec.
template <int TM, int TN>
__device__ __forceinline__ void gemm_store_partial(const mtts_conv_gemm_args &p, f32x16 (&acc)[TM][TN], float *stage,
                                                   float *part, int row0, int col0, int lane) {
    const int M = p.nb * p.To;
    const int lr = lane & 31, lh = lane >> 5, rsub = lane >> 3, c4 = lane & 7;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#pragma unroll
            for (int v = 0; v < 16; ++v) stage[((v & 3) + 8 * (v >> 2) + 4 * lh) * 32 + lr] = acc[i][j][v];
            const int n = col0 + j * 32 + 4 * c4;
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                const float4 x = reinterpret_cast<const float4 *>(stage)[(it * 8 + rsub) * 8 + c4];
                const int m = row0 + i * 32 + it * 8 + rsub;
                if (m < M && n < p.N) *reinterpret_cast<float4 *>(part + (size_t)m * p.N + n) = x;
            }
        }
}

// Epilogue over 16-byte rows: each 32x32 accumulator tile goes through a wave-private 4 KiB LDS
// image (row-major, 32 floats per row -- conflict-free for both the ds_write_b32 of the MFMA layout and
// the ds_read_b128 of the row chunks), then every lane finishes 4 consecutive columns of one row and
// writes them (and reads bias / residual / aux) as float4.  The MFMA layout alone gives each lane one
// column of 16 rows: 4-byte stores in 128-byte row pieces, which left the output-heavy GEMMs (the
// 1024-wide FFN projection, K = 80 linears) running at ~1.5 TB/s.  Needs N, ldc, ldr, ldaux % 4 == 0
// and 16-byte aligned C / C_pre / residual / aux (gemm_epilogue_vec_ok); the caller has retired every
// other use of `stage` (a workgroup barrier after its last LDS read).
__host__ __device__ inline bool gemm_epilogue_vec_ok(const mtts_conv_gemm_args &p) {
    auto al = [](const void *q) { return ((uintptr_t)q & 15) == 0; };
    // (a bf16 C / C_pre / aux row chunk of 4 elements is 8 bytes: 16-byte bases and ld % 4 keep it aligned)
    return p.N % 4 == 0 && p.ldc % 4 == 0 && al(p.C) && al(p.C_pre) && al(p.bias) && (!p.residual || (p.ldr % 4 == 0 && al(p.residual))) &&
           (!p.aux || (p.ldaux % 4 == 0 && al(p.aux)));
}

template <int TM, int TN>
__device__ __forceinline__ void gemm_epilogue_vec(const mtts_conv_gemm_args &p, f32x16 (&acc)[TM][TN], float *stage,
                                                  int row0, int col0, int lane) {
    const int M = p.nb * p.To;
    const float inv_to = 1.0f / (float)p.To;
    const int lr = lane & 31, lh = lane >> 5;
    const bool drop = p.dropout_p > 0.f;
    uint32_t s0 = 0, s1 = 0;
    if (drop) {
        s0 = p.seed[0];
        s1 = p.seed[1];
    }
    const float keep_scale = drop ? 1.0f / (1.0f - p.dropout_p) : 1.0f;
    const int rsub = lane >> 3, c4 = lane & 7;  // this lane's row within an 8-row slab and its column chunk
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        // output rows of the 4 slabs this lane finishes in tile row i (same for every j)
        int crow[4];
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int m = row0 + i * 32 + it * 8 + rsub;
            int b, u;
            divmod_fast(m, p.To, inv_to, b, u);
            crow[it] = m < M ? b * p.To_full + u * p.out_stride + p.out_off : -1;
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#pragma unroll
            for (int v = 0; v < 16; ++v) stage[((v & 3) + 8 * (v >> 2) + 4 * lh) * 32 + lr] = acc[i][j][v];
            const int n = col0 + j * 32 + 4 * c4;
            const bool nok = n < p.N;
            float4 bn = make_float4(0.f, 0.f, 0.f, 0.f);
            if (p.bias && nok) bn = *reinterpret_cast<const float4 *>(p.bias + n);
#pragma unroll
            for (int it = 0; it < 4; ++it) {
                float4 x = reinterpret_cast<const float4 *>(stage)[(it * 8 + rsub) * 8 + c4];
                if (crow[it] < 0 || !nok) continue;
                float e[4] = {x.x + bn.x, x.y + bn.y, x.z + bn.z, x.w + bn.w};
                epilogue_row4(p, crow[it], n, e, s0, s1, keep_scale);
            }
        }
    }
}

}  // namespace mtts
