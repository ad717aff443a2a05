// The CFM decoder's time path on gfx950 (decoder.py:33-49 TimeStepEmbeddingNet, :68-86 Resnet1D.mlp):
//     h1 = e W1^T + b1 ; a1 = silu(h1) ; temb = a1 W2^T + b2 ; a2 = mish(temb) ; tp_i = a2 Wt_i^T + bt_i
// (i over the decoder's Resnet1D blocks), forward and backward, fp32 as the reference keeps it.  B rows
// only (the batch): every product is a skinny GEMM whose cost is latency, not FLOPs.  torch ran it as
// 3 addmm + silu + mish + 2 weight / bias concatenations + a transpose copy forward and 6 mm + 3 bias sums
// + mish' + silu' backward (~25 launches, ~0.1 ms per step).  Here one small-GEMM kernel on the exact
// fp32 MFMA (v_mfma_f32_32x32x2_f32) serves all of it:
//   fwd    C[b, n] = sum_k x[b, k] W_i[n, k] + bias_i[n], act(C) stored beside it
//   dgrad  C[b, k] = (sum_i sum_n dy_i[b, n] W_i[n, k]) * act'(pre[b, k])
//   wgrad  C[n, k] = sum_b dy_i[b, n] a[b, k]   (+ db_i[n] = sum_b dy_i[b, n])
// One workgroup per 32 x 32 tile of C; its waves split the reduction (64 indices per wave and pass, all
// loads of a pass issued at once), and wave 0 adds the waves' partial tiles in wave order through LDS:
// a short dependency chain per launch instead of a K-long one, and a fixed summation order (deterministic).
// A matrix table (up to 8 stacked Linear layers sharing the input rows) replaces torch.cat of their weights.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kMaxWaves = 16;
constexpr int kChunk = 64;  // reduction indices per wave and pass: 32 MFMAs of 32x32x2

enum Mode { kFwd = 0, kDgrad = 1, kWgrad = 2 };

struct MatTable {
    const float *W[MTTS_ROWS_MAX_MATS];
    const float *bias[MTTS_ROWS_MAX_MATS];
    float *out[MTTS_ROWS_MAX_MATS];       // fwd: out_i; wgrad: dW_i
    float *out2[MTTS_ROWS_MAX_MATS];      // fwd: act(out_i) (optional); wgrad: db_i (optional)
    const float *dy[MTTS_ROWS_MAX_MATS];  // dgrad / wgrad: dy_i [B, N_i]
    int N[MTTS_ROWS_MAX_MATS];
    int n_off[MTTS_ROWS_MAX_MATS + 1];    // prefix sums of N (dgrad: the stacked reduction index)
    int nmat;
};

__device__ __forceinline__ float act_fwd(int act, float v) {
    if (act == MTTS_ROWS_ACT_SILU) return v / (1.0f + expf(-v));
    if (act == MTTS_ROWS_ACT_MISH) {
        // mish(v) = v tanh(softplus(v)) = v n / (n + 2), n = e^v (e^v + 2); v >= 15: tanh(softplus) == 1 in fp32
        if (v >= 15.f) return v;
        const float e = expf(v), n = e * (e + 2.f);
        return v * n / (n + 2.f);
    }
    return v;
}

__device__ __forceinline__ float act_grad(int act, float v) {
    if (act == MTTS_ROWS_ACT_SILU) {
        const float s = 1.0f / (1.0f + expf(-v));
        return s * (1.0f + v * (1.0f - s));
    }
    if (act == MTTS_ROWS_ACT_MISH) {
        // d/dv [v tanh(sp(v))] = tanh(sp) + v sigmoid(v) (1 - tanh(sp)^2)
        if (v >= 15.f) return 1.f;
        const float e = expf(v), n = e * (e + 2.f), t = n / (n + 2.f), s = e / (1.f + e);
        return t + v * s * (1.f - t * t);
    }
    return 1.f;
}

// Grid: tiles of C (rows = tm tiles of 32, cols as the mode defines), one workgroup each, nw waves.
// Operand fragments of v_mfma_f32_32x32x2_f32: lane l holds A(row l%32, slot l/32) and B(slot l/32,
// col l%32).  Pass index j covers reduction indices r0 + 4j .. r0 + 4j + 3: slot s of MFMA 2j + e takes
// index r0 + 4j + 2s + e (any fixed bijection works: both operands use the same one).
template <int MODE>
__global__ __launch_bounds__(64 * kMaxWaves) void rows_gemm_kernel(MatTable T, const float *__restrict__ x, int B,
                                                                   int K, int act, const float *__restrict__ pre,
                                                                   float *__restrict__ dx, int col_tiles) {
    __shared__ float part[kMaxWaves][16][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int lr = lane & 31, s = lane >> 5;
    // tile -> (row block, column block, matrix)
    const int rt = blockIdx.x / col_tiles, ct = blockIdx.x - rt * col_tiles;
    int mat = 0, m0 = rt * 32, c0 = ct * 32, R = 0;
    if constexpr (MODE == kFwd) {  // rows b, cols n of matrix mat (stacked column tiles), reduce over K
        while (mat + 1 < T.nmat && c0 >= T.n_off[mat + 1]) ++mat;
        c0 -= T.n_off[mat];
        R = K;
    } else if constexpr (MODE == kDgrad) {  // rows b, cols k, reduce over the stacked n
        R = T.n_off[T.nmat];
    } else {  // rows n of matrix mat (stacked row tiles), cols k, reduce over b
        m0 = rt * 32;
        while (mat + 1 < T.nmat && m0 >= T.n_off[mat + 1]) ++mat;
        m0 -= T.n_off[mat];
        R = B;
    }
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.f;
    for (int r0 = wave * kChunk; r0 < R; r0 += nw * kChunk) {
        float a[32], b[32];  // this pass: 16 index pairs x (A, B)
        // dgrad: the pass's matrix (every N_i is a multiple of kChunk: a pass never straddles two)
        int dm = 0;
        if constexpr (MODE == kDgrad) {
            while (dm + 1 < T.nmat && r0 >= T.n_off[dm + 1]) ++dm;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int r = r0 + 4 * j + 2 * s + e;
                const bool ok = r < R;
                float av = 0.f, bv = 0.f;
                if constexpr (MODE == kFwd) {
                    const int row = min(m0 + lr, B - 1), n = c0 + lr;
                    av = ok && m0 + lr < B ? x[(size_t)row * K + r] : 0.f;
                    bv = ok && n < T.N[mat] ? T.W[mat][(size_t)n * K + r] : 0.f;
                } else if constexpr (MODE == kDgrad) {
                    const int rn = r - T.n_off[dm], Nm = T.N[dm];
                    const int row = min(m0 + lr, B - 1), k = c0 + lr;
                    av = ok && m0 + lr < B ? T.dy[dm][(size_t)row * Nm + rn] : 0.f;
                    bv = ok && k < K ? T.W[dm][(size_t)rn * K + k] : 0.f;
                } else {
                    const int n = m0 + lr, k = c0 + lr, Nm = T.N[mat];
                    av = ok && n < Nm ? T.dy[mat][(size_t)r * Nm + n] : 0.f;
                    bv = ok && k < K ? x[(size_t)r * K + k] : 0.f;
                }
                a[2 * j + e] = av;
                b[2 * j + e] = bv;
            }
        }
#pragma unroll
        for (int j = 0; j < 32; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[j], acc, 0, 0, 0);
    }
    // wave order sum of the partial tiles (wave 0 adds waves 1 .. nw-1 in order)
    if (nw > 1) {
        if (wave > 0) {
#pragma unroll
            for (int v = 0; v < 16; ++v) part[wave][v][lane] = acc[v];
        }
        __syncthreads();
        if (wave > 0) return;
        for (int w = 1; w < nw; ++w)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[v] += part[w][v][lane];
    }
    // C(row, col) of acc[v]: row = (v & 3) + 8 (v >> 2) + 4 s, col = lr
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const int row = m0 + (v & 3) + 8 * (v >> 2) + 4 * s, col = c0 + lr;
        if constexpr (MODE == kFwd) {
            const int N = T.N[mat];
            if (row < B && col < N) {
                const float o = acc[v] + (T.bias[mat] ? T.bias[mat][col] : 0.f);
                T.out[mat][(size_t)row * N + col] = o;
                if (T.out2[mat]) T.out2[mat][(size_t)row * N + col] = act_fwd(act, o);
            }
        } else if constexpr (MODE == kDgrad) {
            if (row < B && col < K) {
                const size_t o = (size_t)row * K + col;
                dx[o] = pre ? acc[v] * act_grad(act, pre[o]) : acc[v];
            }
        } else {
            if (row < T.N[mat] && col < K) T.out[mat][(size_t)row * K + col] = acc[v];
        }
    }
    if constexpr (MODE == kWgrad) {  // the bias gradient: column-tile-0 workgroups, fixed b order
        if (ct == 0 && T.out2[mat] && lane < 32 && m0 + lane < T.N[mat]) {
            const int n = m0 + lane, Nm = T.N[mat];
            float sacc = 0.f;
            for (int b = 0; b < B; ++b) sacc += T.dy[mat][(size_t)b * Nm + n];
            T.out2[mat][n] = sacc;
        }
    }
}

int fill_table(MatTable &T, int nmat, const int32_t *N) {
    MTTS_CHECK_ARG(nmat >= 1 && nmat <= MTTS_ROWS_MAX_MATS && N, "rows_linear: 1..8 matrices");
    T.nmat = nmat;
    T.n_off[0] = 0;
    for (int i = 0; i < nmat; ++i) {
        MTTS_CHECK_ARG(N[i] >= 1 && (nmat == 1 || N[i] % kChunk == 0),
                       "rows_linear: stacked matrices need N_i % 64 == 0");
        T.N[i] = N[i];
        T.n_off[i + 1] = T.n_off[i] + (nmat == 1 ? N[i] : N[i]);
    }
    return MTTS_OK;
}

int waves_for(int R) {
    const int w = (R + kChunk - 1) / kChunk;
    return w < 1 ? 1 : (w > kMaxWaves ? kMaxWaves : w);
}

}  // namespace

extern "C" int mtts_rows_linear_fwd(const float *x, int32_t B, int32_t K, int32_t nmat, const float *const *W,
                                    const float *const *bias, const int32_t *N, float *const *out,
                                    float *const *out_act, int32_t act, void *hip_stream) {
    MTTS_CHECK_ARG(x && W && out && B >= 1 && K >= 1, "rows_linear_fwd: bad args");
    MTTS_CHECK_ARG(act >= MTTS_ROWS_ACT_NONE && act <= MTTS_ROWS_ACT_MISH, "rows_linear_fwd: bad act");
    MatTable T{};
    if (int rc = fill_table(T, nmat, N)) return rc;
    int col_tiles = 0;
    for (int i = 0; i < nmat; ++i) {
        MTTS_CHECK_ARG(W[i] && out[i], "rows_linear_fwd: null matrix / output");
        MTTS_CHECK_ARG(nmat == 1 || N[i] % 32 == 0, "rows_linear_fwd: stacked matrices need N_i % 32 == 0");
        T.W[i] = W[i];
        T.bias[i] = bias ? bias[i] : nullptr;
        T.out[i] = out[i];
        T.out2[i] = out_act ? out_act[i] : nullptr;
        col_tiles += (N[i] + 31) / 32;
    }
    if (nmat == 1) T.n_off[1] = col_tiles * 32;  // one matrix: every column tile is its own
    const int rt = (B + 31) / 32;
    hipLaunchKernelGGL(rows_gemm_kernel<kFwd>, dim3(rt * col_tiles), dim3(64 * waves_for(K)), 0,
                       static_cast<hipStream_t>(hip_stream), T, x, B, K, act, nullptr, nullptr, col_tiles);
    return mtts::check_launch("rows_gemm_kernel<fwd>");
}

extern "C" int mtts_rows_linear_bwd(const float *a, const float *pre, int32_t act, int32_t B, int32_t K, int32_t nmat,
                                    const float *const *W, const int32_t *N, const float *const *dy, float *dx,
                                    float *const *dW, float *const *db, void *hip_stream) {
    MTTS_CHECK_ARG(W && dy && B >= 1 && K >= 1, "rows_linear_bwd: bad args");
    MTTS_CHECK_ARG(act >= MTTS_ROWS_ACT_NONE && act <= MTTS_ROWS_ACT_MISH && (act == MTTS_ROWS_ACT_NONE || pre),
                   "rows_linear_bwd: act' needs the pre-activation");
    MTTS_CHECK_ARG(!dW || a, "rows_linear_bwd: dW needs the input rows");
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    MatTable T{};
    if (int rc = fill_table(T, nmat, N)) return rc;
    int row_tiles = 0;
    for (int i = 0; i < nmat; ++i) {
        MTTS_CHECK_ARG(W[i] && dy[i], "rows_linear_bwd: null matrix");
        T.W[i] = W[i];
        T.dy[i] = dy[i];
        T.out[i] = dW ? dW[i] : nullptr;
        T.out2[i] = db ? db[i] : nullptr;
        MTTS_CHECK_ARG(!dW || dW[i], "rows_linear_bwd: null dW");
        row_tiles += (N[i] + 31) / 32;
    }
    if (nmat == 1) T.n_off[1] = N[0];
    const int kt = (K + 31) / 32;
    if (dx) {
        hipLaunchKernelGGL(rows_gemm_kernel<kDgrad>, dim3(((B + 31) / 32) * kt), dim3(64 * waves_for(T.n_off[nmat])), 0,
                           st, T, nullptr, B, K, act, pre, dx, kt);
        if (int rc = mtts::check_launch("rows_gemm_kernel<dgrad>")) return rc;
    }
    if (dW) {
        if (nmat == 1) T.n_off[1] = row_tiles * 32;
        hipLaunchKernelGGL(rows_gemm_kernel<kWgrad>, dim3(row_tiles * kt), dim3(64 * waves_for(B)), 0, st, T, a, B, K,
                           act, nullptr, nullptr, kt);
        if (int rc = mtts::check_launch("rows_gemm_kernel<wgrad>")) return rc;
    }
    return MTTS_OK;
}
