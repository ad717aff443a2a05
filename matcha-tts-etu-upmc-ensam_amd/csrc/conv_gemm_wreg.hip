// Weight-stationary bf16 GEMM for short reductions (round 5): the linears / 1x1 convs with K <= 256 -- the decoder
// FeedForward up-projection and its GELU' dgrad, the stacked q|k|v and out projections, Resnet1D's res_conv --
// behind mtts_conv_gemm (include/mtts_decoder.h), schedule ids MTTS_GEMM_WREG + i.
//
// Why: the LDS-DMA kernels (conv_gemm_glds.hip) restream the packed weights through LDS for every 64-row tile;
// the round-5 fill probe (tools/r5/fill_probe.hip) puts L2 -> LDS at ~75 GB/s per CU, so W -- two bf16 planes
// under the parity policy -- is most of what bounds them.  Here a wave owns 32 output columns and holds their
// whole K <= 256 reduction as MFMA B fragments in VGPRs (16 x 4 registers per plane), loaded once; the
// workgroup (4 waves, 128 columns) walks its 32-row tiles of A, which alone stream through an LDS ring by
// LDS-DMA and are read by all four waves.  Per tile a wave issues K / 16 (x planes) MFMAs against one A
// fragment read each; two workgroups per CU overlap one's epilogue with the other's MFMAs.
// Numerics: per output element the MFMAs run in the K order of conv_gemm_glds_kernel's unsplit launches (16-wide
// sub-steps ascending, hi plane before lo plane) -- bitwise equal to them (tests/test_gemm_wreg_gpu.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <utility>

#include "conv_gemm_wreg.h"
#include "gemm_epilogue.h"
#include "lds_dma.h"
#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
using mtts::f32x16;
using mtts::u32x4;

constexpr int kNW = 4, kNT = 64 * kNW;  // 4 waves x 32 columns = 128 columns per workgroup
constexpr int kBM = 32;                  // rows per A tile
constexpr int kKMax = 256;
constexpr uint32_t kOob = mtts::kDmaOob;

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

// A image of one tile: kBM rows padded to kKMax elements (512 B bf16 / 1 KiB fp32 per row); 16-byte chunk c of row r
// at c ^ (r & 15) (bf16) / 32-byte unit u at u ^ (r & 15) (fp32): the 16-lane groups of the fragment reads spread
// over the banks
template <bool ABF16>
struct WrGeom {
    static constexpr int ES = ABF16 ? 2 : 4;
    static constexpr int ROW = kKMax * ES;                // bytes per image row
    static constexpr int TILE = kBM * ROW;                // 16 / 32 KiB
    static constexpr int INS = TILE / 1024;               // 1 KiB DMA pieces per tile
    static constexpr int PER_WAVE = INS / kNW;            // 4 / 8
    static constexpr int S = ABF16 ? 3 : 2;               // ring stages
    static constexpr int LDS = S * TILE + kNW * 4096;     // + the per-wave epilogue images
    static_assert(INS % kNW == 0, "tile pieces");
};

template <bool ABF16, int NPL, int KS, int EK, bool ROWMASK>
__global__ __launch_bounds__(kNT, 2) void conv_gemm_wreg_kernel(mtts_conv_gemm_args p, int ncg, int mtiles) {
    using G = WrGeom<ABF16>;
    constexpr int ES = G::ES, S = G::S;
    __shared__ __attribute__((aligned(1024))) unsigned char sst[S * G::TILE];
    __shared__ __attribute__((aligned(16))) float sepi[kNW * 1024];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, lh = lane >> 5;
    const int M = p.nb * p.To;
    // workgroup -> (column group, row stream); the R workgroups of a column group take its 32-row tiles
    // round robin
    const int nwg = gridDim.x, R = nwg / ncg;
    const int g = mtts::xcd_relabel(blockIdx.x, nwg);
    const int cg = g % ncg, r = g / ncg;
    const int n0 = cg * (32 * kNW) + 32 * wave;  // this wave's 32 columns
    const int ntl = r < mtiles ? (mtiles - 1 - r) / R + 1 : 0;

    // ---- W: the wave's 32 columns x K as B fragments, every plane (lane: column n0 + lr, k = 16 s + 8 lh .. + 8)
    bf16x8 wf[NPL][KS];
    {
        const int n = n0 + lr;
        const bool nok = n < p.N;
        const uint16_t *wb = static_cast<const uint16_t *>(p.W) + (size_t)(nok ? n : 0) * p.Kp + 8 * lh;
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const uint4 v = nok ? *reinterpret_cast<const uint4 *>(wb + (size_t)pl * p.N * p.Kp + 16 * s)
                                    : make_uint4(0u, 0u, 0u, 0u);
                wf[pl][s] = __builtin_bit_cast(bf16x8, v);
            }
    }
    // retire the W loads here: left pending into the tile loop, the compiler's wait for them (merged over the loop's
    // back edge) became a vmcnt(0) at the loop head that drained every A prefetch of every tile
    mtts::wait_vmcnt<0>();

    // ---- A tiles by LDS-DMA: piece q = wave * PER_WAVE + i of a tile is 1 KiB = 2 (bf16) / 1 (fp32) image rows.
    // A row = GEMM row (one tap, stride 1, no offset); a_scale is applied in the epilogue (ROWMASK), so no
    // compiler-visible load sits between the DMAs (its wait would drain them)
    const u32x4 rsa = mtts::make_rsrc(p.A, (uint32_t)((long long)M * p.lda * ES));
    const uint32_t lds0 = mtts::lds_addr(sst);
    auto issue = [&](int ti, int stage) {  // tile index ti of this workgroup (>= ntl: zeros, unused)
        const int m0 = (r + ti * R) * kBM;
        const bool tv = ti < ntl;
#pragma unroll
        for (int i = 0; i < G::PER_WAVE; ++i) {
            const int q = wave * G::PER_WAVE + i;
            constexpr int RPI = 1024 / G::ROW;  // image rows per piece
            const int row = q * RPI + lane / (64 / RPI);
            const int slot = lane % (64 / RPI);  // 16-byte slot within the image row
            int c;                               // logical 16-byte chunk of the row it holds
            if constexpr (ABF16) c = slot ^ (row & 15);
            else c = ((slot >> 1) ^ (row & 15)) * 2 + (slot & 1);
            const int m = m0 + row;
            const uint32_t vo = tv && m < M && c * (16 / ES) < p.K
                                    ? (uint32_t)(((long long)m * p.lda + c * (16 / ES)) * ES)
                                    : kOob;
            mtts::bload16(vo, rsa, 0u, __builtin_amdgcn_readfirstlane(lds0 + stage * G::TILE + q * 1024));
        }
    };

    for (int s0 = 0; s0 < S - 1; ++s0) issue(s0, s0);

    int cur = 0;
    for (int ti = 0; ti < ntl; ++ti) {
        mtts::wait_vmcnt<G::PER_WAVE * (S - 2)>();  // this wave's pieces of tile ti have landed ...
        mtts::lds_barrier();                        // ... and everyone's; tile ti - 1's reads are done
        issue(ti + S - 1, cur == 0 ? S - 1 : cur - 1);
        const unsigned char *sa = sst + cur * G::TILE;
        f32x16 acc;
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[v] = 0.f;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            bf16x8 af;
            if constexpr (ABF16) {
                const int c = 2 * s + lh;
                af = *reinterpret_cast<const bf16x8 *>(sa + lr * G::ROW + ((c ^ (lr & 15)) << 4));
            } else {
                const int u = 2 * s + lh;  // 32-byte unit: 8 fp32
                const unsigned char *src = sa + lr * G::ROW + ((u ^ (lr & 15)) << 5);
                const float4 x0 = *reinterpret_cast<const float4 *>(src);
                const float4 x1 = *reinterpret_cast<const float4 *>(src + 16);
                af = __builtin_bit_cast(bf16x8, make_uint4(pack2(x0.x, x0.y), pack2(x0.z, x0.w), pack2(x1.x, x1.y),
                                                           pack2(x1.z, x1.w)));
            }
#pragma unroll
            for (int pl = 0; pl < NPL; ++pl) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, wf[pl][s], acc, 0, 0, 0);
        }
        f32x16 a1[1][1];
        a1[0][0] = acc;
        mtts::gemm_epilogue_vec_v<8, 1, 1, EK, ROWMASK>(p, a1, sepi + wave * 1024, (r + ti * R) * kBM, n0, lane);
        cur = cur == S - 1 ? 0 : cur + 1;
    }
    mtts::wait_vmcnt<0>();  // no DMA may still target this workgroup's LDS when it retires
}

struct WrGrid {
    int ncg, mtiles, R;  // column groups, 32-row tiles, row streams per column group
};

WrGrid wreg_grid(const mtts_conv_gemm_args &p, int M) {
    static const int cus = [] {
        int dev = 0, n = 256;
        hipDeviceProp_t pr;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&pr, dev) == hipSuccess && pr.multiProcessorCount > 0)
            n = pr.multiProcessorCount;
        return n;
    }();
    static const int per_cu = [] {  // MTTS_WREG_WG_PER_CU: workgroups per CU of the grid (default 2)
        const char *e = getenv("MTTS_WREG_WG_PER_CU");
        return e && atoi(e) > 0 ? atoi(e) : 2;
    }();
    WrGrid g;
    g.ncg = (p.N + 32 * kNW - 1) / (32 * kNW);
    g.mtiles = (M + kBM - 1) / kBM;
    g.R = std::max(1, std::min(g.mtiles, (cus * per_cu) / g.ncg));
    return g;
}

template <bool ABF16, int NPL, int KS, int EK, bool ROWMASK>
int launch_wreg_e(const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    static_assert(WrGeom<ABF16>::LDS <= 80 * 1024, "two workgroups per CU");
    const WrGrid g = wreg_grid(p, M);
    hipLaunchKernelGGL((conv_gemm_wreg_kernel<ABF16, NPL, KS, EK, ROWMASK>), dim3((unsigned)(g.ncg * g.R)), dim3(kNT),
                       0, st, p, g.ncg, g.mtiles);
    return mtts::check_launch("conv_gemm_wreg_kernel");
}

template <bool ABF16, int NPL, int KS>
int launch_wreg_t(const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    const bool rm = p.a_scale != nullptr;
    static const bool rt_only = [] { const char *e = getenv("MTTS_WREG_EK_RT"); return e && e[0] == '1'; }();
    switch (rt_only ? (int)mtts::EK_RT : mtts::gemm_epilogue_kind(p)) {
        case mtts::EK_LIN_C16:
            return rm ? launch_wreg_e<ABF16, NPL, KS, mtts::EK_LIN_C16, true>(p, M, st)
                      : launch_wreg_e<ABF16, NPL, KS, mtts::EK_LIN_C16, false>(p, M, st);
        case mtts::EK_LIN_C32:
            return rm ? launch_wreg_e<ABF16, NPL, KS, mtts::EK_LIN_C32, true>(p, M, st)
                      : launch_wreg_e<ABF16, NPL, KS, mtts::EK_LIN_C32, false>(p, M, st);
        case mtts::EK_GELU:
            return rm ? launch_wreg_e<ABF16, NPL, KS, mtts::EK_GELU, true>(p, M, st)
                      : launch_wreg_e<ABF16, NPL, KS, mtts::EK_GELU, false>(p, M, st);
        case mtts::EK_DGELU:
            return rm ? launch_wreg_e<ABF16, NPL, KS, mtts::EK_DGELU, true>(p, M, st)
                      : launch_wreg_e<ABF16, NPL, KS, mtts::EK_DGELU, false>(p, M, st);
        default:
            return rm ? launch_wreg_e<ABF16, NPL, KS, mtts::EK_RT, true>(p, M, st)
                      : launch_wreg_e<ABF16, NPL, KS, mtts::EK_RT, false>(p, M, st);
    }
}

template <bool ABF16, int NPL>
int launch_wreg_k(const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    switch (p.K / 16) {
        case 16: return launch_wreg_t<ABF16, NPL, 16>(p, M, st);
        case 12: return launch_wreg_t<ABF16, NPL, 12>(p, M, st);
        case 10: return launch_wreg_t<ABF16, NPL, 10>(p, M, st);
        case 5: return launch_wreg_t<ABF16, NPL, 5>(p, M, st);
        default: return mtts::fail(MTTS_ERR_UNSUPPORTED, "conv_gemm: weight-stationary schedule: K not instantiated");
    }
}

}  // namespace

namespace mtts {

// K in {80, 160, 192, 256}; one tap at stride 1 (A row = output row: linears and 1x1 convs); bf16 MFMA on one
// or two weight planes; bf16 or fp32 A with 16-byte aligned rows; a 0/1 row mask or none; the 16-byte epilogue
bool conv_gemm_wreg_applies(const mtts_conv_gemm_args &p) {
    const int ks = p.K / 16;
    if (p.K % 16 || p.K > kKMax || !(ks == 16 || ks == 12 || ks == 10 || ks == 5)) return false;
    if (p.ntaps != 1 || p.cin != p.K || p.in_stride != 1 || p.off[0] != 0 || p.Ti != p.To) return false;
    if (p.flags & (MTTS_GEMM_F_A_SPLIT | MTTS_GEMM_F_SPLIT3)) return false;
    if (p.a_scale && !(p.flags & MTTS_GEMM_F_BINARY_SCALE)) return false;
    const bool a16 = p.flags & MTTS_GEMM_F_A_BF16;
    const int es = a16 ? 2 : 4, npl = (p.flags & MTTS_GEMM_F_W_SPLIT) ? 2 : 1;
    if (p.lda % (16 / es) || (uintptr_t)p.A % 16 || (uintptr_t)p.W % 16 || p.Kp % 8) return false;
    if ((long long)p.nb * p.Ti * p.lda * es >= (1ll << 31) - (1ll << 20)) return false;
    if ((long long)npl * p.N * p.Kp >= (1ll << 31)) return false;
    // the kernel always finishes 8 columns per lane (gemm_epilogue_vec_v<8>): N % 8 == 4 would write past the row
    return gemm_epilogue_vec_ok(p) && gemm_epilogue_vec8_ok(p);
}

bool conv_gemm_wreg_preferred(const mtts_conv_gemm_args &p, int M) {
    const WrGrid g = wreg_grid(p, M);
    return g.mtiles >= 2 * g.R || g.mtiles == g.R;
}

int conv_gemm_wreg_launch(const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    const bool a16 = p.flags & MTTS_GEMM_F_A_BF16, w2 = p.flags & MTTS_GEMM_F_W_SPLIT;
    if (a16) return w2 ? launch_wreg_k<true, 2>(p, M, st) : launch_wreg_k<true, 1>(p, M, st);
    return w2 ? launch_wreg_k<false, 2>(p, M, st) : launch_wreg_k<false, 1>(p, M, st);
}

}  // namespace mtts
