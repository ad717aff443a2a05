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
                              ? val * dropout_scale(p.dropout_p)
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

// V (4 or 8) consecutive bf16 values from / to 16-byte-aligned memory as one uint2 / uint4 access
template <int V>
__device__ __forceinline__ void store_bf16v(void *dst, const float (&e)[V]) {
    typedef float f32x2_ __attribute__((ext_vector_type(2)));
    typedef __bf16 bf16x2_ __attribute__((ext_vector_type(2)));
    uint32_t w[V / 2];
#pragma unroll
    for (int q = 0; q < V / 2; ++q)
        w[q] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_){e[2 * q], e[2 * q + 1]}, bf16x2_));
    if constexpr (V == 4) *reinterpret_cast<uint2 *>(dst) = make_uint2(w[0], w[1]);
    else *reinterpret_cast<uint4 *>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
}
template <int V>
__device__ __forceinline__ void load_bf16v(const void *src, float (&a)[V]) {  // bf16 -> fp32 is exact
    uint32_t w[V / 2];
    if constexpr (V == 4) {
        const uint2 h = *reinterpret_cast<const uint2 *>(src);
        w[0] = h.x, w[1] = h.y;
    } else {
        const uint4 h = *reinterpret_cast<const uint4 *>(src);
        w[0] = h.x, w[1] = h.y, w[2] = h.z, w[3] = h.w;
    }
#pragma unroll
    for (int q = 0; q < V / 2; ++q) {
        a[2 * q] = __uint_as_float(w[q] << 16);
        a[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
}
template <int V>
__device__ __forceinline__ void load_f32v(const float *src, float (&a)[V]) {
#pragma unroll
    for (int q = 0; q < V / 4; ++q) {
        const float4 x = reinterpret_cast<const float4 *>(src)[q];
        a[4 * q] = x.x, a[4 * q + 1] = x.y, a[4 * q + 2] = x.z, a[4 * q + 3] = x.w;
    }
}
template <int V>
__device__ __forceinline__ void store_f32v(float *dst, const float (&e)[V]) {
#pragma unroll
    for (int q = 0; q < V / 4; ++q)
        reinterpret_cast<float4 *>(dst)[q] = make_float4(e[4 * q], e[4 * q + 1], e[4 * q + 2], e[4 * q + 3]);
}

// Epilogue kinds fixed at compile time (EK > 0: the weight-stationary kernel classifies each launch on the host,
// mtts::gemm_epilogue_kind): the per-element tests of p.act / p.flags / null pointers become constants and the
// branches drop out.  EK_RT reads everything at run time (every other caller).
enum : int {
    EK_RT = 0,
    EK_LIN_C16 = 1,  // no activation, C bf16; bias / dropout / residual / c_scale at run time; no C_pre
    EK_LIN_C32 = 2,  // the same with an fp32 C
    EK_GELU = 3,     // fast GELU, bf16 C_pre and C; bias / dropout at run time; no residual / c_scale
    EK_DGELU = 4,    // fast GELU' on a bf16 aux, bf16 C; bias / dropout at run time; no C_pre / residual / c_scale
    EK_RELU32 = 5,   // ReLU, fp32 C; bias / dropout / residual / c_scale at run time; no C_pre (the text encoder's FFN)
    EK_DRELU32 = 6,  // ReLU' on an fp32 aux, fp32 C; the same run-time terms; no C_pre (its backward)
};

// -DMTTS_EK_RELU=0: the ReLU / ReLU' launches keep the run-time epilogue (A/B builds)
#ifndef MTTS_EK_RELU
#define MTTS_EK_RELU 1
#endif
__host__ __device__ inline int gemm_epilogue_kind(const mtts_conv_gemm_args &p) {
    const bool fast = p.flags & MTTS_GEMM_F_FAST_ACT, pre16 = p.flags & MTTS_GEMM_F_PRE_BF16,
               c16 = p.flags & MTTS_GEMM_F_C_BF16;
    if (p.act == MTTS_ACT_NONE && !p.C_pre) return c16 ? EK_LIN_C16 : EK_LIN_C32;
    if (p.act == MTTS_ACT_GELU && fast && pre16 && c16 && p.C_pre && !p.residual && !p.c_scale) return EK_GELU;
    if (p.act == MTTS_ACT_DGELU && fast && pre16 && c16 && !p.C_pre && p.aux && !p.residual && !p.c_scale)
        return EK_DGELU;
#if MTTS_EK_RELU
    if (p.act == MTTS_ACT_RELU && !p.C_pre && !c16) return EK_RELU32;
    if (p.act == MTTS_ACT_DRELU && !p.C_pre && !c16 && !pre16 && p.aux) return EK_DRELU32;
#endif
    return EK_RT;
}

// Everything after the bias for V (4 or 8) consecutive columns n.. of output row crow (16-byte I/O: V = 8
// writes a bf16 C / C_pre as one dwordx4 per lane -- the dwordx2 stores of V = 4 are issue-bound at about
// half the bytes per cycle, MI355X_MICROARCH.md's epilogue store-tail row).
template <int V, int EK = EK_RT>
__device__ __forceinline__ void epilogue_rowv(const mtts_conv_gemm_args &p, int crow, int n, float (&e)[V],
                                              uint32_t s0, uint32_t s1, float keep_scale) {
    constexpr bool RT = EK == EK_RT;
    constexpr bool RELU = EK == EK_RELU32 || EK == EK_DRELU32;
    const int act = RT ? p.act
                       : EK == EK_GELU ? MTTS_ACT_GELU
                       : EK == EK_DGELU ? MTTS_ACT_DGELU
                       : EK == EK_RELU32 ? MTTS_ACT_RELU
                       : EK == EK_DRELU32 ? MTTS_ACT_DRELU : MTTS_ACT_NONE;
    const bool fast = RT ? (p.flags & MTTS_GEMM_F_FAST_ACT) != 0 : true;
    const bool pre16 = RT ? (p.flags & MTTS_GEMM_F_PRE_BF16) != 0 : EK != EK_DRELU32;
    const bool c16 = RT ? (p.flags & MTTS_GEMM_F_C_BF16) != 0 : EK != EK_LIN_C32 && !RELU;
    const bool has_pre = RT ? p.C_pre != nullptr : EK == EK_GELU;
    const bool has_drop = p.dropout_p > 0.f;
    const bool has_res = (RT || EK == EK_LIN_C16 || EK == EK_LIN_C32 || RELU) && p.residual;
    const bool has_cs = (RT || EK == EK_LIN_C16 || EK == EK_LIN_C32 || RELU) && p.c_scale;
    const size_t off = (size_t)crow * p.ldc + n;
    if (has_pre) {
        if (pre16) store_bf16v<V>(reinterpret_cast<uint16_t *>(p.C_pre) + off, e);
        else store_f32v<V>(p.C_pre + off, e);
    }
    if (act) {
        float av[V];
#pragma unroll
        for (int q = 0; q < V; ++q) av[q] = 0.f;
        if (act == MTTS_ACT_DGELU || act == MTTS_ACT_DRELU) {
            const size_t ao = (size_t)crow * p.ldaux + n;
            if (pre16) load_bf16v<V>(reinterpret_cast<const uint16_t *>(p.aux) + ao, av);
            else load_f32v<V>(p.aux + ao, av);
        }
#pragma unroll
        for (int q = 0; q < V; ++q) e[q] = epi_act(act, e[q], &av[q], fast);
    }
    if (has_drop) {
#pragma unroll
        for (int q = 0; q < V; ++q)
            e[q] = dropout_keep(s0, s1, (uint32_t)crow, (uint32_t)(n + q), p.dropout_p) ? e[q] * keep_scale : 0.f;
    }
    if (has_res) {
        float r[V];
        load_f32v<V>(p.residual + (size_t)crow * p.ldr + n, r);
#pragma unroll
        for (int q = 0; q < V; ++q) e[q] += r[q];
    }
    if (has_cs) {
        const float cs = p.c_scale[crow];
#pragma unroll
        for (int q = 0; q < V; ++q) e[q] *= cs;
    }
    if (c16) store_bf16v<V>(reinterpret_cast<uint16_t *>(p.C) + off, e);
    else store_f32v<V>(p.C + off, e);
}

__device__ __forceinline__ void epilogue_row4(const mtts_conv_gemm_args &p, int crow, int n, float (&e)[4],
                                              uint32_t s0, uint32_t s1, float keep_scale) {
    epilogue_rowv<4>(p, crow, n, e, s0, s1, keep_scale);
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

// 8 columns per lane (16-byte bf16 stores) when N, ldc and a bf16 aux row are multiples of 8
__host__ __device__ inline bool gemm_epilogue_vec8_ok(const mtts_conv_gemm_args &p) {
    return p.N % 8 == 0 && p.ldc % 8 == 0 && (!p.aux || p.ldaux % 8 == 0);
}

// EK: epilogue kind (above); ROWMASK: zero the accumulators of the rows whose a_scale is 0 (a one-tap GEMM that
// did not mask its A rows: A row = GEMM row)
template <int V, int TM, int TN, int EK = EK_RT, bool ROWMASK = false>
__device__ __forceinline__ void gemm_epilogue_vec_v(const mtts_conv_gemm_args &p, f32x16 (&acc)[TM][TN], float *stage,
                                                    int row0, int col0, int lane) {
    constexpr int L = 32 / V, RP = 64 / L;  // lanes per 32-column row; rows per pass
    const int M = p.nb * p.To;
    const float inv_to = 1.0f / (float)p.To;
    const int lr = lane & 31, lh = lane >> 5;
    const bool drop = p.dropout_p > 0.f;
    uint32_t s0 = 0, s1 = 0;
    if (drop) {
        s0 = p.seed[0];
        s1 = p.seed[1];
    }
    const float keep_scale = drop ? dropout_scale(p.dropout_p) : 1.0f;
    const int rsub = lane / L, cv = lane % L;  // this lane's row within an RP-row slab and its column chunk
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        // output rows of the slabs this lane finishes in tile row i (same for every j)
        int crow[32 / RP];
        bool live[32 / RP];
#pragma unroll
        for (int it = 0; it < 32 / RP; ++it) {
            const int m = row0 + i * 32 + it * RP + rsub;
            int b, u;
            divmod_fast(m, p.To, inv_to, b, u);
            crow[it] = m < M ? b * p.To_full + u * p.out_stride + p.out_off : -1;
            live[it] = true;
            if (ROWMASK && m < M) live[it] = p.a_scale[m] != 0.f;
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#pragma unroll
            for (int v = 0; v < 16; ++v) stage[((v & 3) + 8 * (v >> 2) + 4 * lh) * 32 + lr] = acc[i][j][v];
            const int n = col0 + j * 32 + V * cv;
            const bool nok = n < p.N;
            float bn[V];
#pragma unroll
            for (int q = 0; q < V; ++q) bn[q] = 0.f;
            if (p.bias && nok) load_f32v<V>(p.bias + n, bn);
#pragma unroll
            for (int it = 0; it < 32 / RP; ++it) {
                float e[V];
                load_f32v<V>(stage + (it * RP + rsub) * 32 + V * cv, e);
                if (crow[it] < 0 || !nok) continue;
#pragma unroll
                for (int q = 0; q < V; ++q) e[q] = (live[it] ? e[q] : 0.f) + bn[q];
                epilogue_rowv<V, EK>(p, crow[it], n, e, s0, s1, keep_scale);
            }
        }
    }
}

// The kind is classified once per call (wave-uniform) and each kind runs its own compile-time-specialised
// epilogue: the generic one spent ~300 scalar instructions per 32 x 32 tile re-testing p.act / p.flags / null
// pointers (PMC SQ_INSTS_SALU, profiles/r05/wreg/pmc_ff1_first/); specialised, the weight-stationary kernel's
// launches ran 13 % faster (964 vs 1114 us per step, profiles/r05/wreg/replay_ek_*.jsonl).
template <int TM, int TN>
__device__ __forceinline__ void gemm_epilogue_vec(const mtts_conv_gemm_args &p, f32x16 (&acc)[TM][TN], float *stage,
                                                  int row0, int col0, int lane) {
    if (!gemm_epilogue_vec8_ok(p)) {
        gemm_epilogue_vec_v<4>(p, acc, stage, row0, col0, lane);
        return;
    }
    switch (gemm_epilogue_kind(p)) {
        case EK_LIN_C16: gemm_epilogue_vec_v<8, TM, TN, EK_LIN_C16>(p, acc, stage, row0, col0, lane); break;
        case EK_LIN_C32: gemm_epilogue_vec_v<8, TM, TN, EK_LIN_C32>(p, acc, stage, row0, col0, lane); break;
        case EK_GELU: gemm_epilogue_vec_v<8, TM, TN, EK_GELU>(p, acc, stage, row0, col0, lane); break;
        case EK_DGELU: gemm_epilogue_vec_v<8, TM, TN, EK_DGELU>(p, acc, stage, row0, col0, lane); break;
        case EK_RELU32: gemm_epilogue_vec_v<8, TM, TN, EK_RELU32>(p, acc, stage, row0, col0, lane); break;
        case EK_DRELU32: gemm_epilogue_vec_v<8, TM, TN, EK_DRELU32>(p, acc, stage, row0, col0, lane); break;
        default: gemm_epilogue_vec_v<8, TM, TN, EK_RT>(p, acc, stage, row0, col0, lane); break;
    }
}

}  // namespace mtts
