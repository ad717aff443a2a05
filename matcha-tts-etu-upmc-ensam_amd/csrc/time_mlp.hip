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
#include <cstdlib>

#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kChunk = 64;  // reduction indices per wave and pass: 32 MFMAs of 32x32x2

enum Mode { kFwd = 0, kDgrad = 1, kWgrad = 2 };

struct MatTable {
    const float *W[MTTS_ROWS_MAX_MATS];
    const float *bias[MTTS_ROWS_MAX_MATS];
    float *out[MTTS_ROWS_MAX_MATS];       // fwd: out_i; wgrad: dW_i
    float *out2[MTTS_ROWS_MAX_MATS];      // fwd: act(out_i) (optional); wgrad: db_i (optional)
    const float *dy[MTTS_ROWS_MAX_MATS];  // dgrad / wgrad: dy_i [B, N_i]
    int N[MTTS_ROWS_MAX_MATS];
    int n_off[MTTS_ROWS_MAX_MATS + 1];    // prefix sums of N_i rounded up to 32 (the stacked 32-wide tiles)
    int r_off[MTTS_ROWS_MAX_MATS + 1];    // prefix sums of N_i rounded up to 64 (dgrad's reduction index:
                                          // a wave's 64 indices never straddle two matrices)
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

// One workgroup = one 32 x 32 tile of C and one 256-wide range of the reduction (4 waves x 64); the
// reduction is split over KS workgroups per tile so that a launch spreads over ~200 CUs.  Operand fragments
// of v_mfma_f32_32x32x2_f32: lane l holds A(row l%32, slot l/32) and B(slot l/32, col l%32); within a
// wave's 64 indices, slot s of MFMA j takes index 32 s + j (one fixed bijection for both operands).
// Operands contiguous along the reduction (x / W rows in the forward, dy rows in dgrad) are staged through
// LDS with coalesced float4 loads (a 32 x 64 block per wave); the others are read straight into the
// fragment (lanes run along their contiguous dimension).  The 4 wave partials are added in wave order;
// with KS > 1 the workgroup stores its partial tile and the LAST of the tile's KS workgroups to arrive
// (a per-tile ticket counter, agent-scope release / acquire) adds the KS partials in index order and runs
// the epilogue -- a fixed summation order whatever the arrival order, and the counter is reset for the next
// launch (graph replays reuse it).
constexpr int kWaves = 4;
constexpr int kRange = kWaves * kChunk;  // reduction indices per workgroup
constexpr int kLd = 65;                  // staged row pitch (floats): conflict-free column reads

struct Ws {
    float *part;        // [tiles][KS][32 * 32]
    unsigned *counter;  // [tiles], zero between launches
    int ks;
    int passes;         // kRange-wide passes per workgroup (the waves accumulate across them)
};

template <int MODE>
__global__ __launch_bounds__(64 * kWaves) void rows_gemm_kernel(MatTable T, const float *__restrict__ x, int B, int K,
                                                                int act, const float *__restrict__ pre,
                                                                float *__restrict__ dx, int col_tiles, Ws ws) {
    extern __shared__ float lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lr = lane & 31, s = lane >> 5;
    const int tile = blockIdx.x / ws.ks, ksi = blockIdx.x - tile * ws.ks;
    const int rt = tile / col_tiles, ct = tile - rt * col_tiles;
    int mat = 0, m0 = rt * 32, c0 = ct * 32, R = 0;
    if constexpr (MODE == kFwd) {  // rows b, cols n of matrix mat (stacked column tiles), reduce over K
        while (mat + 1 < T.nmat && c0 >= T.n_off[mat + 1]) ++mat;
        c0 -= T.n_off[mat];
        R = K;
    } else if constexpr (MODE == kDgrad) {  // rows b, cols k, reduce over the stacked n
        R = T.r_off[T.nmat];
    } else {  // rows n of matrix mat (stacked row tiles), cols k, reduce over b
        while (mat + 1 < T.nmat && m0 >= T.n_off[mat + 1]) ++mat;
        m0 -= T.n_off[mat];
        R = B;
    }
    float *sA = lds + wave * 2 * 32 * kLd, *sB = sA + 32 * kLd;
    // stage a 32 x 64 block (rows row0.., indices r0..r0+63) of a row-major matrix, zero outside
    auto stage = [&](const float *base, int ld, int nrows, int r0, int r_end, float *dst) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = q * 64 + lane, row = e >> 4, c4 = (e & 15) * 4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (row < nrows && r0 + c4 < r_end) v = *reinterpret_cast<const float4 *>(base + (size_t)row * ld + r0 + c4);
            dst[row * kLd + c4] = v.x;
            dst[row * kLd + c4 + 1] = v.y;
            dst[row * kLd + c4 + 2] = v.z;
            dst[row * kLd + c4 + 3] = v.w;
        }
    };
    f32x16 acc;
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[v] = 0.f;
    for (int pass = 0; pass < ws.passes; ++pass) {
        const int r0 = (ksi * ws.passes + pass) * kRange + wave * kChunk;  // this wave's 64 indices
        if (pass > 0) __syncthreads();  // every wave has read the previous pass's staged blocks
        float a[32], b[32];
        if constexpr (MODE == kFwd) {
            stage(x + (size_t)m0 * K, K, min(32, B - m0), r0, R, sA);
            stage(T.W[mat] + (size_t)c0 * K, K, min(32, T.N[mat] - c0), r0, R, sB);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                a[j] = sA[lr * kLd + 32 * s + j];
                b[j] = sB[lr * kLd + 32 * s + j];
            }
        } else if constexpr (MODE == kDgrad) {
            int dm = 0;  // the wave's matrix (r_off: a wave's 64 indices never straddle two)
            while (dm + 1 < T.nmat && r0 >= T.r_off[dm + 1]) ++dm;
            const int base = T.r_off[dm], Nm = T.N[dm];
            stage(T.dy[dm] + (size_t)m0 * Nm - base, Nm, min(32, B - m0), r0, min(R, base + Nm), sA);
            __syncthreads();
            const int k = c0 + lr;
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                const int r = r0 + 32 * s + j;
                a[j] = sA[lr * kLd + 32 * s + j];
                b[j] = r - base < Nm && k < K ? T.W[dm][(size_t)(r - base) * K + k] : 0.f;
            }
        } else {
            const int n = m0 + lr, k = c0 + lr, Nm = T.N[mat];
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                const int r = r0 + 32 * s + j;
                a[j] = r < R && n < Nm ? T.dy[mat][(size_t)r * Nm + n] : 0.f;
                b[j] = r < R && k < K ? x[(size_t)r * K + k] : 0.f;
            }
        }
#pragma unroll
        for (int j = 0; j < 32; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[j], acc, 0, 0, 0);
    }
    // the workgroup's tile: waves 1..3 through LDS (the staging area is free after this barrier), wave order
    const int nw = blockDim.x >> 6;
    if (nw > 1) {
        __syncthreads();
        float *part = lds;  // [nw][16][64]
        if (wave > 0) {
#pragma unroll
            for (int v = 0; v < 16; ++v) part[(wave * 16 + v) * 64 + lane] = acc[v];
        }
        __syncthreads();
        if (wave > 0) return;
        for (int w = 1; w < nw; ++w)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[v] += part[(w * 16 + v) * 64 + lane];
    }
    if (ws.ks > 1) {  // split reduction: the last workgroup of the tile to arrive sums the partials in order
        float *mine = ws.part + ((size_t)tile * ws.ks + ksi) * 1024;
#pragma unroll
        for (int v = 0; v < 16; ++v) mine[v * 64 + lane] = acc[v];
        __threadfence();  // release: the partial is visible device-wide before the ticket
        unsigned ticket = 0;
        if (lane == 0) ticket = atomicAdd(ws.counter + tile, 1u);
        ticket = __shfl(ticket, 0);
        if (ticket != (unsigned)ws.ks - 1) return;
        __threadfence();  // acquire: the other workgroups' partials
        const float *all = ws.part + (size_t)tile * ws.ks * 1024;
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[v] = __builtin_nontemporal_load(all + v * 64 + lane);
        for (int q = 1; q < ws.ks; ++q)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[v] += __builtin_nontemporal_load(all + (size_t)q * 1024 + v * 64 + lane);
        if (lane == 0) atomicExch(ws.counter + tile, 0u);  // ready for the next launch
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
            for (int b2 = 0; b2 < B; ++b2) sacc += T.dy[mat][(size_t)b2 * Nm + n];
            T.out2[mat][n] = sacc;
        }
    }
}

int fill_table(MatTable &T, int nmat, const int32_t *N) {
    MTTS_CHECK_ARG(nmat >= 1 && nmat <= MTTS_ROWS_MAX_MATS && N, "rows_linear: 1..8 matrices");
    T.nmat = nmat;
    T.n_off[0] = T.r_off[0] = 0;
    for (int i = 0; i < nmat; ++i) {
        MTTS_CHECK_ARG(N[i] >= 1, "rows_linear: N_i >= 1");
        T.N[i] = N[i];
        T.n_off[i + 1] = T.n_off[i] + (N[i] + 31) / 32 * 32;
        T.r_off[i + 1] = T.r_off[i] + (N[i] + kChunk - 1) / kChunk * kChunk;
    }
    return MTTS_OK;
}

// launch geometry of one rows GEMM: KS workgroups per tile, waves per workgroup, dynamic LDS bytes
struct Geo {
    int ks, waves, passes;
    size_t lds;
};
// passes per workgroup: MTTS_ROWS_PASSES (default 1: the whole reduction split over workgroups)
int passes_of(int R) {
    const char *e = getenv("MTTS_ROWS_PASSES");
    const int want = e ? atoi(e) : 1, need = (R + kRange - 1) / kRange;
    return want < 1 ? 1 : (want > need ? need : want);
}

Geo geometry(int R, bool staged) {
    Geo g;
    g.passes = passes_of(R);
    g.ks = (R + kRange * g.passes - 1) / (kRange * g.passes);
    g.waves = R >= kRange ? kWaves : (R + kChunk - 1) / kChunk;
    const size_t stage = staged ? (size_t)g.waves * 2 * 32 * kLd * sizeof(float) : 0;
    const size_t red = g.waves > 1 ? (size_t)g.waves * 16 * 64 * sizeof(float) : 0;
    g.lds = stage > red ? stage : red;
    return g;
}

int check_ws(const Geo &g, int tiles, void *ws, size_t ws_bytes, Ws &w) {
    w.ks = g.ks;
    w.passes = g.passes;
    w.part = nullptr;
    w.counter = nullptr;
    if (g.ks == 1) return MTTS_OK;
    const size_t need = mtts::align_up((size_t)tiles * sizeof(unsigned), 256) + (size_t)tiles * g.ks * 1024 * sizeof(float);
    if (!ws || ws_bytes < need || (uintptr_t)ws % 256)
        return mtts::fail(MTTS_ERR_WORKSPACE, "rows_linear: workspace too small (mtts_rows_linear_workspace_size)");
    w.counter = static_cast<unsigned *>(ws);
    w.part = reinterpret_cast<float *>(static_cast<char *>(ws) + mtts::align_up((size_t)tiles * sizeof(unsigned), 256));
    return MTTS_OK;
}

}  // namespace

extern "C" size_t mtts_rows_linear_workspace_size(int32_t B, int32_t K, int32_t nmat, const int32_t *N) {
    if (B < 1 || K < 1 || nmat < 1 || nmat > MTTS_ROWS_MAX_MATS || !N) return 0;
    size_t nt = 0, nr = 0;  // 32-column tiles of the stacked outputs; dgrad's padded reduction length
    for (int i = 0; i < nmat; ++i) {
        nt += (size_t)(N[i] + 31) / 32;
        nr += (size_t)(N[i] + kChunk - 1) / kChunk * kChunk;
    }
    const size_t rt = (size_t)(B + 31) / 32, kt = (size_t)(K + 31) / 32;
    auto ks = [](size_t r) { return (r + kRange - 1) / kRange; };
    // (tiles, splits) of the forward, dgrad and wgrad launches
    const size_t t[3] = {rt * nt, rt * kt, nt * kt}, k[3] = {ks(K), ks(nr), ks(B)};
    size_t tiles = 0, parts = 0;
    for (int m = 0; m < 3; ++m) {
        if (k[m] < 2) continue;
        tiles = t[m] > tiles ? t[m] : tiles;
        parts = t[m] * k[m] > parts ? t[m] * k[m] : parts;
    }
    return mtts::align_up(tiles * sizeof(unsigned), 256) + parts * 1024 * sizeof(float);
}

extern "C" int mtts_rows_linear_fwd(const float *x, int32_t B, int32_t K, int32_t nmat, const float *const *W,
                                    const float *const *bias, const int32_t *N, float *const *out,
                                    float *const *out_act, int32_t act, void *workspace, size_t workspace_bytes,
                                    void *hip_stream) {
    MTTS_CHECK_ARG(x && W && out && B >= 1 && K >= 4 && K % 4 == 0 && (uintptr_t)x % 16 == 0,
                   "rows_linear_fwd: bad args (K % 4 == 0, 16-byte aligned rows)");
    MTTS_CHECK_ARG(act >= MTTS_ROWS_ACT_NONE && act <= MTTS_ROWS_ACT_MISH, "rows_linear_fwd: bad act");
    MatTable T{};
    if (int rc = fill_table(T, nmat, N)) return rc;
    int col_tiles = 0;
    for (int i = 0; i < nmat; ++i) {
        MTTS_CHECK_ARG(W[i] && out[i] && (uintptr_t)W[i] % 16 == 0, "rows_linear_fwd: null / unaligned matrix");
        T.W[i] = W[i];
        T.bias[i] = bias ? bias[i] : nullptr;
        T.out[i] = out[i];
        T.out2[i] = out_act ? out_act[i] : nullptr;
        col_tiles += (N[i] + 31) / 32;
    }
    const int tiles = ((B + 31) / 32) * col_tiles;
    const Geo g = geometry(K, true);
    Ws w;
    if (int rc = check_ws(g, tiles, workspace, workspace_bytes, w)) return rc;
    hipLaunchKernelGGL(rows_gemm_kernel<kFwd>, dim3(tiles * g.ks), dim3(64 * g.waves), g.lds,
                       static_cast<hipStream_t>(hip_stream), T, x, B, K, act, nullptr, nullptr, col_tiles, w);
    return mtts::check_launch("rows_gemm_kernel<fwd>");
}

extern "C" int mtts_rows_linear_bwd(const float *a, const float *pre, int32_t act, int32_t B, int32_t K, int32_t nmat,
                                    const float *const *W, const int32_t *N, const float *const *dy, float *dx,
                                    float *const *dW, float *const *db, void *workspace, size_t workspace_bytes,
                                    void *hip_stream) {
    MTTS_CHECK_ARG(W && dy && B >= 1 && K >= 1, "rows_linear_bwd: bad args");
    MTTS_CHECK_ARG(act >= MTTS_ROWS_ACT_NONE && act <= MTTS_ROWS_ACT_MISH && (act == MTTS_ROWS_ACT_NONE || pre),
                   "rows_linear_bwd: act' needs the pre-activation");
    MTTS_CHECK_ARG(!dW || a, "rows_linear_bwd: dW needs the input rows");
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    MatTable T{};
    if (int rc = fill_table(T, nmat, N)) return rc;
    int row_tiles = 0;
    for (int i = 0; i < nmat; ++i) {
        MTTS_CHECK_ARG(W[i] && dy[i] && (!dx || (N[i] % 4 == 0 && (uintptr_t)dy[i] % 16 == 0)),
                       "rows_linear_bwd: null matrix (dx: N_i % 4 == 0, 16-byte aligned dy rows)");
        T.W[i] = W[i];
        T.dy[i] = dy[i];
        T.out[i] = dW ? dW[i] : nullptr;
        T.out2[i] = db ? db[i] : nullptr;
        MTTS_CHECK_ARG(!dW || dW[i], "rows_linear_bwd: null dW");
        row_tiles += (N[i] + 31) / 32;
    }
    const int kt = (K + 31) / 32;
    if (dx) {
        const int tiles = ((B + 31) / 32) * kt;
        const Geo g = geometry(T.r_off[nmat], true);
        Ws w;
        if (int rc = check_ws(g, tiles, workspace, workspace_bytes, w)) return rc;
        hipLaunchKernelGGL(rows_gemm_kernel<kDgrad>, dim3(tiles * g.ks), dim3(64 * g.waves), g.lds, st, T, nullptr, B,
                           K, act, pre, dx, kt, w);
        if (int rc = mtts::check_launch("rows_gemm_kernel<dgrad>")) return rc;
    }
    if (dW) {
        const Geo g = geometry(B, false);
        Ws w;
        if (int rc = check_ws(g, row_tiles * kt, workspace, workspace_bytes, w)) return rc;
        hipLaunchKernelGGL(rows_gemm_kernel<kWgrad>, dim3(row_tiles * kt * g.ks), dim3(64 * g.waves), g.lds, st, T, a,
                           B, K, act, nullptr, nullptr, kt, w);
        if (int rc = mtts::check_launch("rows_gemm_kernel<wgrad>")) return rc;
    }
    return MTTS_OK;
}
