// "A-resident" implicit GEMM for the bf16 decoder path (gfx950 MFMA).
//
// Same contract as conv_gemm_kernel (mtts_conv_gemm_args, include/mtts_decoder.h); different schedule,
// chosen because the decoder's GEMMs are small-K (256..1536) and latency-bound when A is re-streamed
// per K step:
//   * a block owns BM = 32 consecutive output rows u0..u0+31 of ONE batch element b, so the input rows
//     all its taps touch form one contiguous panel  [u0*in_stride + min_off, (u0+31)*in_stride + max_off].
//     The panel (R rows x cin channels) is loaded ONCE, in one burst (every load in flight together),
//     masked (a_scale) and converted to bf16 into LDS;
//   * only W streams: [BN=256][32] bf16 tiles through a register ring two steps deep + two LDS buffers,
//     one barrier per K step; W is small and stays in L2;
//   * the block loops over N in 256-wide chunks reusing the panel, so A is read from HBM exactly once;
//     blockIdx.y splits N chunks across blocks when that is needed to fill the chip;
//   * 4 waves, wave w owns columns [64w, 64w+64) of the chunk: two 32x32x16 MFMA tiles per K substep.
// LDS rows are padded by 16 bytes: (cin+8)/2 dwords per panel row and 20 dwords per W row make the
// 16-lane ds_read_b128 fragment reads conflict-free for stride-1 gathers (2-way for stride 2).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBM = 32;
constexpr int kBN = 256;
constexpr int kBK = 32;
constexpr int kThreads = 256;
constexpr int kWPad = 8;                     // bf16 elements of padding per W LDS row
constexpr int kWLd = kBK + kWPad;            // 40 -> 80-byte rows
constexpr int kWChunks = kBN * kBK / 8 / kThreads;  // 16-byte W chunks per thread per K step (= 4)

typedef float f32x2p __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2p __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float a, float b) {  // one v_cvt_pk_bf16_f32
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2p){a, b}, bf16x2p));
}

struct PanelGeom {
    int min_off, span, R, ld;  // panel rows R, LDS row length ld (bf16 elements)
};

__host__ __device__ inline PanelGeom panel_geom(const mtts_conv_gemm_args &p) {
    int mn = p.off[0], mx = p.off[0];
    for (int j = 1; j < p.ntaps; ++j) {
        mn = p.off[j] < mn ? p.off[j] : mn;
        mx = p.off[j] > mx ? p.off[j] : mx;
    }
    PanelGeom g;
    g.min_off = mn;
    g.span = mx - mn;
    g.R = (kBM - 1) * p.in_stride + g.span + 1;
    g.ld = p.cin + 8;
    return g;
}

__host__ __device__ inline size_t panel_lds_bytes(const mtts_conv_gemm_args &p) {
    const PanelGeom g = panel_geom(p);
    return (size_t)g.R * g.ld * 2 + (size_t)2 * kBN * kWLd * 2;
}

__global__ __launch_bounds__(kThreads, 2) void conv_gemm_panel_kernel(mtts_conv_gemm_args p, int tiles_per_b,
                                                                   int chunks_per_block) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    const PanelGeom g = panel_geom(p);
    uint16_t *panel = lds;                                        // [R][ld]
    uint16_t *wbuf = lds + (size_t)g.R * g.ld;                     // [2][kBN][kWLd]
    // keep the W buffers 16-byte aligned: R*ld*2 is a multiple of 16 because ld % 8 == 0

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 31, lh = lane >> 5;
    const int b = blockIdx.x / tiles_per_b;
    const int u0 = (blockIdx.x - b * tiles_per_b) * kBM;
    const int nrows = min(kBM, p.To - u0);
    const int r_lo = u0 * p.in_stride + g.min_off;  // input row (within batch b) of panel row 0

    // ---- panel: R x cin fp32 -> masked bf16, all loads of a thread issued before any store ----
    {
        const int c4 = p.cin / 4;
        const int total = g.R * c4;
        for (int base = 0; base < total; base += 4 * kThreads) {
            float4 v[4];
            float sc[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int idx = base + i * kThreads + tid;
                const int r = idx / c4, c = (idx - r * c4) * 4;
                const int ir = r_lo + r;
                v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
                sc[i] = 0.f;
                if (idx < total && ir >= 0 && ir < p.Ti) {
                    const size_t row = (size_t)b * p.Ti + ir;
                    v[i] = *reinterpret_cast<const float4 *>(p.A + row * p.lda + c);
                    sc[i] = p.a_scale ? p.a_scale[row] : 1.f;
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int idx = base + i * kThreads + tid;
                if (idx < total) {
                    const int r = idx / c4, c = (idx - r * c4) * 4;
                    uint2 w;
                    w.x = pack2(v[i].x * sc[i], v[i].y * sc[i]);
                    w.y = pack2(v[i].z * sc[i], v[i].w * sc[i]);
                    *reinterpret_cast<uint2 *>(panel + (size_t)r * g.ld + c) = w;
                }
            }
        }
    }

    const int nk = (p.K + kBK - 1) / kBK;
    const int nchunks = (p.N + kBN - 1) / kBN;
    const int c_begin = blockIdx.y * chunks_per_block;
    const int c_end = min(nchunks, c_begin + chunks_per_block);
    uint32_t s0 = 0, s1 = 0;
    if (p.dropout_p > 0.f) {
        s0 = p.seed[0];
        s1 = p.seed[1];
    }

    // W staging assignment: chunk q -> row q>>2, k-offset (q&3)*8
    int w_row[kWChunks], w_kc[kWChunks];
#pragma unroll
    for (int c = 0; c < kWChunks; ++c) {
        const int q = tid + kThreads * c;
        w_row[c] = q >> 2;
        w_kc[c] = (q & 3) * 8;
    }

    for (int ch = c_begin; ch < c_end; ++ch) {
        const int n0 = ch * kBN;
        uint4 ra[kWChunks], rb[kWChunks];
        auto load_w = [&](uint4 (&r)[kWChunks], int kt) {
            const int k0 = kt * kBK;
#pragma unroll
            for (int c = 0; c < kWChunks; ++c) {
                const int n = n0 + w_row[c], k = k0 + w_kc[c];
                r[c] = (n < p.N && k < p.Kp)
                           ? *reinterpret_cast<const uint4 *>(static_cast<const uint16_t *>(p.W) + (size_t)n * p.Kp + k)
                           : make_uint4(0, 0, 0, 0);
            }
        };
        auto store_w = [&](const uint4 (&r)[kWChunks], int buf) {
#pragma unroll
            for (int c = 0; c < kWChunks; ++c)
                *reinterpret_cast<uint4 *>(wbuf + ((size_t)buf * kBN + w_row[c]) * kWLd + w_kc[c]) = r[c];
        };

        f32x16 acc[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[j][v] = 0.f;

        // A fragment of K substep ks: this lane's 8 consecutive K indices kk = k0 + 16ks + 8lh live in
        // tap j = kk / cin at channel kk % cin, panel row lr*in_stride + off_j - min_off.  (j, c) are
        // tracked incrementally per substep (+32 per K step): no division in the loop.
        int tj[2], tc[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int kk = ks * 16 + 8 * lh;
            tj[ks] = kk / p.cin;
            tc[ks] = kk - tj[ks] * p.cin;
        }
        auto compute = [&](int buf, int kt) {
            const int k0 = kt * kBK;
#pragma unroll
            for (int ks = 0; ks < kBK / 16; ++ks) {
                const int kk = k0 + ks * 16 + 8 * lh;
                bf16x8 af;
                if (kk < p.K) {
                    const int prow = lr * p.in_stride + mtts::tap_off(p, tj[ks]) - g.min_off;
                    af = *reinterpret_cast<const bf16x8 *>(panel + (size_t)prow * g.ld + tc[ks]);
                } else {
                    af = bf16x8{};
                }
                tc[ks] += kBK;
                while (tc[ks] >= p.cin) { tc[ks] -= p.cin; ++tj[ks]; }
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const bf16x8 bfr = *reinterpret_cast<const bf16x8 *>(
                        wbuf + ((size_t)buf * kBN + wave * 64 + t * 32 + lr) * kWLd + ks * 16 + 8 * lh);
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, acc[t], 0, 0, 0);
                }
            }
        };

        __syncthreads();  // panel ready / previous chunk's last W reads done
        load_w(ra, 0);
        store_w(ra, 0);
        if (nk > 1) load_w(rb, 1);
        __syncthreads();
        for (int kt = 0; kt < nk; kt += 2) {
            if (kt + 2 < nk) load_w(ra, kt + 2);
            compute(0, kt);
            if (kt + 1 < nk) store_w(rb, 1);
            __syncthreads();
            if (kt + 1 >= nk) break;
            if (kt + 3 < nk) load_w(rb, kt + 3);
            compute(1, kt + 1);
            if (kt + 2 < nk) store_w(ra, 0);
            __syncthreads();
        }

        // ---- epilogue: rows u0 + r of batch b.  64-bit bases are block-uniform; in-tile offsets are
        // small 32-bit values (r < 32), so nothing 64-bit per row is kept live across N chunks ----
        const size_t row0 = (size_t)b * p.To_full + (size_t)u0 * p.out_stride + p.out_off;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int n = n0 + wave * 64 + t * 32 + lr;
            if (n >= p.N) continue;
            const float bn = p.bias ? p.bias[n] : 0.f;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int r = (v & 3) + 8 * (v >> 2) + 4 * lh;
                if (r >= nrows) continue;
                const int dr = r * p.out_stride;
                float val = acc[t][v] + bn;
                if (p.C_pre) p.C_pre[row0 * p.ldc + dr * p.ldc + n] = val;
                if (p.act) val = mtts::epi_act(p.act, val, p.aux + row0 * p.ldaux + dr * p.ldaux + n);
                if (p.dropout_p > 0.f)
                    val = mtts::dropout_keep(s0, s1, (uint32_t)row0 + (uint32_t)dr, (uint32_t)n, p.dropout_p)
                              ? val * (1.0f / (1.0f - p.dropout_p))
                              : 0.f;
                if (p.residual) val += p.residual[row0 * p.ldr + dr * p.ldr + n];
                if (p.c_scale) val *= p.c_scale[row0 + dr];
                p.C[row0 * p.ldc + dr * p.ldc + n] = val;
            }
        }
    }
}

}  // namespace

namespace mtts {

// Launches the panel kernel when it applies (bf16, panel fits LDS); returns 1 if it did not apply.
int conv_gemm_panel_launch(const mtts_conv_gemm_args &p, hipStream_t st) {
    const size_t lds = panel_lds_bytes(p);
    if (lds > 150 * 1024) return 1;
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(conv_gemm_panel_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return 1;
        attr_set = true;
    }
    const int tiles_per_b = (p.To + kBM - 1) / kBM;
    const int nblocks_m = p.nb * tiles_per_b;
    const int nchunks = (p.N + kBN - 1) / kBN;
    // split N chunks across blocks until the grid has >= 2 blocks per CU (or every chunk is its own block)
    int cpb = nchunks;
    while (cpb > 1 && (long)nblocks_m * ((nchunks + cpb - 1) / cpb) < 512) cpb = (cpb + 1) / 2;
    dim3 grid(nblocks_m, (nchunks + cpb - 1) / cpb);
    hipLaunchKernelGGL(conv_gemm_panel_kernel, grid, dim3(kThreads), lds, st, p, tiles_per_b, cpb);
    return 0;
}

}  // namespace mtts
