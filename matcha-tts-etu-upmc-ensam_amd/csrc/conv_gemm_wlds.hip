// Weight-resident bf16 implicit GEMM (round 6): the decoder's k = 1 / 2 / 3 convs and linears with K <= 768 --
// Resnet1D's Block1D convs, the transposed conv's phases, their dgrads, the q|k|v dgrad -- behind mtts_conv_gemm
// (include/mtts_decoder.h), schedule id MTTS_GEMM_WLDS.
//
// Why: the LDS-DMA kernels (conv_gemm_glds.hip) stream the packed weights through LDS again for every 64-row tile.
// On the decoder's 256-column convs that is most of what a workgroup loads (W 256 x 768 x 2 B per tile per plane
// against 64 x 768 x 2 B of A), and the per-CU L2 -> LDS fill (~70 GB/s, MI355X_MICROARCH.md 'gather into LDS';
// round-5 fill probe) bounds them at 0.13 of HBM / 5 % of MFMA peak.  Here a workgroup owns 64 weight rows -- 64
// output columns (one plane) or 32 columns x two planes (the parity policy's split weights) -- over the whole
// reduction K <= 768: 96 KiB of LDS, loaded ONCE; it then walks its 128-row tiles and only A streams.  A k = 3 conv
// stages each tile's input rows once (130 rows for 128 outputs) and reads them at the three tap offsets, so A is
// not re-read per tap either.  Per 128-row tile the workgroup moves ~66 KiB (bf16 A, 256 channels) for 25 MFLOP.
//
// Layout: row-major LDS images with XOR-swizzled 16-byte chunks (a_swz / w_swz), conflict-free fragment reads at any
// row shift.  The K loop runs over 64-byte channel chunks of the staged rows (32 bf16 / 16 fp32 channels: "steps"),
// tap-major inside a step; steps of consecutive tiles form one pipeline, S = 5 stages deep (~36 KiB in flight: an
// LDS-DMA fill takes ~1.5 us from issue to landing, so the bytes in flight, not the instruction count, set the
// rate), and the next tile's first chunks are in flight during a tile's epilogue.  (The first version's chunk-major
// images -- 64 rows x 16 bytes per DMA instruction -- and 3 stages of 9 KiB ran each step at ~14 GB/s per CU.)
// Validity: a staged input row outside [0, nb * Ti) or whose 0/1 mask is 0 is DMA'd as zeros (per-tile lane bits,
// computed for ALL of the workgroup's tiles in the prologue: no mask load inside the DMA pipeline, whose wait would
// drain it); a tap that falls outside its utterance reads the stage's zero row instead.
// Numerics: fp32 accumulation of bf16 products in (channel chunk, tap, 16-channel substep) order -- not bitwise the
// LDS-DMA kernels' tap-major order; within fp32 accumulation error of them (tests/test_gemm_wlds_gpu.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

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

constexpr int kNW = 4, kNT = 64 * kNW;  // 4 waves, each 32 output rows of the 128-row tile
constexpr int kBM = 32 * kNW;           // rows per tile
constexpr int kKMax = 768;              // the W image: 64 rows x K bf16, chunk-major
constexpr int kMaxTiles = 8;            // tiles per workgroup (validity bits precomputed for all of them)
constexpr uint32_t kOob = mtts::kDmaOob;

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

// NTAP taps at stride 1: a tile's staged input rows NR = 128 + NTAP - 1 (+ a zero row when a tap can leave its
// utterance), NRP rounded to 16 rows = NI one-KiB DMA instructions per stage (16 rows x 64 bytes each), wave w
// issuing instructions w, w + 4, ... (PWV(w) of them); rows past NR are DMA'd from out of range: zeros
template <int NTAP>
struct WlGeom {
    static constexpr int NR = kBM + NTAP - 1;
    static constexpr int NRP = (NR + (NTAP > 1 ? 1 : 0) + 15) / 16 * 16;
    static constexpr int NI = NRP / 16;
    static constexpr int PW = (NI + kNW - 1) / kNW;  // the most any wave issues per stage
    static constexpr int STAGE = NI * 1024;
    static constexpr int pwv(int w) { return (NI - w + kNW - 1) / kNW; }
};

// counted wait for wave w: its DMAs of the last `steps` issued pipeline steps may stay in flight
template <int NTAP, int STEPS>
__device__ __forceinline__ void wait_steps(int wave) {
    using G = WlGeom<NTAP>;
    if (wave == 0) mtts::wait_vmcnt<G::pwv(0) * STEPS>();
    else if (wave == 1) mtts::wait_vmcnt<G::pwv(1) * STEPS>();
    else if (wave == 2) mtts::wait_vmcnt<G::pwv(2) * STEPS>();
    else mtts::wait_vmcnt<G::pwv(3) * STEPS>();
}

// LDS images, row-major with 16-byte chunks XOR-swizzled so that 16 lanes reading one logical chunk of 16
// consecutive rows hit distinct banks: A rows are 64 bytes (chunk c of row r at c ^ ((r >> 2) & 3)), W rows are
// K * 2 bytes (chunk c at c ^ (row & 15) inside its aligned group of 16).  The DMA fills 16 A rows (4 lanes per row:
// 64 contiguous source bytes) or 1 KiB of W rows (contiguous) per wave instruction.
__device__ __forceinline__ int a_swz(int row, int c) { return row * 64 + ((c ^ ((row >> 2) & 3)) << 4); }
__device__ __forceinline__ int w_swz(int row, int c) { return ((c & ~15) | ((c & 15) ^ (row & 15))) << 4; }

template <bool ABF16, int NPL, int NTAP, int S, int EK>
__global__ __launch_bounds__(kNT, 1) void conv_gemm_wlds_kernel(mtts_conv_gemm_args p, int ncg, int mtiles, int off_min, int dbg) {
    using G = WlGeom<NTAP>;
    constexpr int ES = ABF16 ? 2 : 4;
    constexpr int CPC = 64 / ES;         // channels per staged 64-byte row (one pipeline step)
    constexpr int SUB = CPC / 16;        // 16-channel MFMA substeps per step
    constexpr int TN = NPL == 2 ? 1 : 2; // 32-column accumulator blocks per wave
    constexpr int NRP = G::NRP, PW = G::PW, NI = G::NI;
    __shared__ __attribute__((aligned(1024))) unsigned char sw[64 * kKMax * 2];
    __shared__ __attribute__((aligned(1024))) unsigned char sa[S * G::STAGE];
    __shared__ __attribute__((aligned(16))) float sepi[kNW * 1024];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, lh = lane >> 5;
    const int M = p.nb * p.To, K = p.K, cin = p.cin;
    const int nch = cin / CPC;  // steps per tile
    const int nwg = gridDim.x, R = nwg / ncg;
    const int g = mtts::xcd_relabel(blockIdx.x, nwg);
    const int cg = g % ncg, r = g / ncg;
    const int n0 = cg * (NPL == 2 ? 32 : 64);
    const int ntl = r < mtiles ? (mtiles - 1 - r) / R + 1 : 0;
    const int nsteps = ntl * nch;
    const int arows = p.nb * p.Ti;  // Ti == To (stride 1): input row of output row m at tap offset o is m + o
    // the bias of this lane's accumulator columns, loaded now and added to the finished accumulators (the same fp32
    // add the epilogue does): an epilogue load would wait for -- drain -- the DMAs in flight behind it
    float bias[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + 32 * j + lr;
        bias[j] = p.bias && n < p.N ? p.bias[n] : 0.f;
    }
    // the epilogue's arguments with every stream it could load made compile-time absent (conv_gemm_wlds_applies
    // refuses them): no load, and no wait for one, can sit in the tile loop
    mtts_conv_gemm_args pe = p;
    pe.bias = nullptr;
    pe.residual = nullptr;
    pe.c_scale = nullptr;
    pe.aux = nullptr;
    pe.C_pre = nullptr;
    pe.seed = nullptr;
    pe.dropout_p = 0.f;

    // ---- per-tile staging validity (bit i * PW + k: this lane's row of DMA instruction k of tile i), all tiles
    // now: the mask loads are retired before the first DMA is issued
    uint32_t vbits = 0;
    for (int i = 0; i < ntl; ++i) {
        const int m0 = (r + i * R) * kBM;
#pragma unroll
        for (int k = 0; k < PW; ++k) {
            const int q = wave + kNW * k;
            const int row = 16 * q + (lane >> 2);
            const int gr = m0 + off_min + row;
            bool v = q < NI && row < G::NR && gr >= 0 && gr < arows;
            if (v && p.a_scale) v = p.a_scale[gr] != 0.f;
            vbits |= (uint32_t)v << (i * PW + k);
        }
    }
    // retire the bias / mask loads here: left pending, the compiler's wait before their first use (the first
    // tile's epilogue) is a vmcnt(0) that would also drain the DMAs in flight by then
    mtts::wait_vmcnt<0>();

    // ---- W image: 64 rows x K bf16, row w = plane * 32 + column (two planes) or column; instruction q fills bytes
    // 1024 q .. of the image
    const u32x4 rsw = mtts::make_rsrc(p.W, (uint32_t)((long long)NPL * p.N * p.Kp * 2));
    {
        const uint32_t lw = mtts::lds_addr(sw);
        const int cpr = K / 8;  // 16-byte chunks per W row
        for (int q = wave; q < K / 8; q += kNW) {
            const int t = 64 * q + lane, w = t / cpr, pc = t - w * cpr;
            const int c = (pc & ~15) | ((pc & 15) ^ (w & 15));
            const int pl = NPL == 2 ? w >> 5 : 0, n = n0 + (NPL == 2 ? w & 31 : w);
            const uint32_t vw = n < p.N ? (uint32_t)((((long long)pl * p.N + n) * p.Kp + c * 8) * 2) : kOob;
            mtts::bload16(vw, rsw, 0u, __builtin_amdgcn_readfirstlane(lw + q * 1024));
        }
    }

    // ---- A staging: instruction q of a stage fills image rows 16 q .. 16 q + 15 (lane: row 16 q + lane / 4, slot
    // lane % 4 <- logical chunk (lane % 4) ^ ((row >> 2) & 3))
    const u32x4 rsa = mtts::make_rsrc(p.A, (uint32_t)((long long)arows * p.lda * ES));
    const uint32_t la0 = mtts::lds_addr(sa);
    uint32_t av[PW];  // this lane's source byte offsets for the current issue tile (channel chunk 0)
    int atile = -1;
    auto issue = [&](int st, int stage) {
        if (st >= nsteps) return;
        const int ti = st / nch, ch = st - ti * nch;
        if (ti != atile) {
            atile = ti;
            const int m0 = (r + ti * R) * kBM;
#pragma unroll
            for (int k = 0; k < PW; ++k) {
                const int q = wave + kNW * k;
                const int row = 16 * q + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 3);
                const bool v = (vbits >> (ti * PW + k)) & 1u;
                av[k] = v ? (uint32_t)(((long long)(m0 + off_min + row) * p.lda + c * (16 / ES)) * ES) : kOob;
            }
        }
        const uint32_t soff = (uint32_t)(ch * CPC * ES);
        if (dbg & 2) return;  // diagnostic: no A staging
#pragma unroll
        for (int k = 0; k < PW; ++k) {
            const int q = wave + kNW * k;
            if (q < NI)  // wave-uniform
                mtts::bload16(av[k], rsa, soff, __builtin_amdgcn_readfirstlane(la0 + stage * G::STAGE + q * 1024));
        }
    };

    // ---- per-lane fragment rows of the current compute tile: image row of output row 32 * wave + lr at tap j, or
    // the zero row when the tap leaves the utterance
    int arow[NTAP];
    auto tile_rows = [&](int ti) {
        const int m = (r + ti * R) * kBM + 32 * wave + lr;
        int b = 0, u = 0;
        mtts::divmod_fast(m < M ? m : 0, p.To, 1.0f / (float)p.To, b, u);
#pragma unroll
        for (int j = 0; j < NTAP; ++j) {
            const int o = p.off[0] + j * (NTAP > 1 ? p.off[1] - p.off[0] : 0);
            const int ui = u + o;
            const bool v = ui >= 0 && ui < p.Ti;
            arow[j] = v ? 32 * wave + lr + (o - off_min) : NRP - 1;
        }
    };

    for (int s0 = 0; s0 < S - 1; ++s0) issue(s0, s0);

    const int wrow0 = lr * K * 2, wrow1 = (32 + lr) * K * 2;  // this lane's two W rows (w & 15 == lr & 15)
    int cur = 0, st = 0;
    for (int ti = 0; ti < ntl; ++ti) {
        tile_rows(ti);
        // the tile's accumulators live only inside its chunk loop (loop-carried across tiles, the register
        // allocator copied them out of the AGPRs at every step, behind a vmcnt(0) that drained the DMAs in flight)
        f32x16 acc[1][TN];
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[0][j][v] = 0.f;
        for (int ch = 0; ch < nch; ++ch, ++st) {
            // steps issued after st: min(S - 2, nsteps - 1 - st); W's loads are all older than step 0's
            if (st + S - 2 < nsteps) wait_steps<NTAP, S - 2>(wave);
            else mtts::wait_vmcnt<0>();
            mtts::lds_barrier();
            issue(st + S - 1, cur == 0 ? S - 1 : cur - 1);
            const unsigned char *sb = sa + cur * G::STAGE;
            // every fragment of the step is read first, then the MFMAs run back to back: with one wave per SIMD
            // nothing else hides an LDS read, and read-MFMA pairs exposed its latency at every MFMA
            bf16x8 af[NTAP][SUB], bw[NTAP][SUB][2];
#pragma unroll
            for (int j = 0; j < NTAP; ++j) {
#pragma unroll
                for (int s = 0; s < SUB; ++s) {
                    if constexpr (ABF16) {
                        af[j][s] = *reinterpret_cast<const bf16x8 *>(sb + a_swz(arow[j], 2 * s + lh));
                    } else {
                        const float4 x0 = *reinterpret_cast<const float4 *>(sb + a_swz(arow[j], 2 * lh));
                        const float4 x1 = *reinterpret_cast<const float4 *>(sb + a_swz(arow[j], 2 * lh + 1));
                        af[j][s] = __builtin_bit_cast(bf16x8, make_uint4(pack2(x0.x, x0.y), pack2(x0.z, x0.w),
                                                                         pack2(x1.x, x1.y), pack2(x1.z, x1.w)));
                    }
                    // W chunk of k = j * cin + ch * CPC + 16 s + 8 lh
                    const int cw = (j * cin + ch * CPC + 16 * s) / 8 + lh;
                    const int so = w_swz(lr, cw);
                    bw[j][s][0] = *reinterpret_cast<const bf16x8 *>(sw + wrow0 + so);
                    bw[j][s][1] = *reinterpret_cast<const bf16x8 *>(sw + wrow1 + so);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            if (dbg & 1) {  // diagnostic: reads, no MFMAs (keep the reads alive)
#pragma unroll
                for (int j = 0; j < NTAP; ++j)
#pragma unroll
                    for (int s = 0; s < SUB; ++s) acc[0][0][0] += (float)af[j][s][0] + (float)bw[j][s][0][1] + (float)bw[j][s][1][2];
            } else
#pragma unroll
            for (int j = 0; j < NTAP; ++j) {
#pragma unroll
                for (int s = 0; s < SUB; ++s) {
                    if constexpr (NPL == 2) {
                        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[j][s], bw[j][s][0], acc[0][0], 0, 0, 0);
                        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[j][s], bw[j][s][1], acc[0][0], 0, 0, 0);
                    } else {
                        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[j][s], bw[j][s][0], acc[0][0], 0, 0, 0);
                        acc[0][TN - 1] =
                            __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[j][s], bw[j][s][1], acc[0][TN - 1], 0, 0, 0);
                    }
                }
            }
            cur = cur == S - 1 ? 0 : cur + 1;
        }
        if (p.bias) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[0][j][v] += bias[j];
        }
        // (no global load in this epilogue -- conv_gemm_wlds_applies refuses residual / c_scale / dropout: its
        // wait would drain the DMAs in flight)
        mtts::gemm_epilogue_vec_v<8, 1, TN, EK, false>(pe, acc, sepi + wave * 1024, (r + ti * R) * kBM + 32 * wave, n0,
                                                       lane);
    }
    mtts::wait_vmcnt<0>();  // no DMA may still target this workgroup's LDS when it retires
}

struct WlGrid {
    int ncg, mtiles, R;
};

WlGrid wlds_grid(const mtts_conv_gemm_args &p, int M) {
    static const int cus = [] {
        int dev = 0, n = 256;
        hipDeviceProp_t pr;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&pr, dev) == hipSuccess && pr.multiProcessorCount > 0)
            n = pr.multiProcessorCount;
        return n;
    }();
    const int npl = (p.flags & MTTS_GEMM_F_W_SPLIT) ? 2 : 1;
    WlGrid g;
    g.ncg = (p.N + (npl == 2 ? 31 : 63)) / (npl == 2 ? 32 : 64);
    g.mtiles = (M + kBM - 1) / kBM;
    g.R = std::max(1, std::min(g.mtiles, cus / g.ncg));
    // every stream's tiles must fit the precomputed validity bits
    g.R = std::max(g.R, (g.mtiles + kMaxTiles - 1) / kMaxTiles);
    return g;
}

template <bool ABF16, int NPL, int NTAP, int EK>
int launch_wlds_e(const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    constexpr int S = 5;
    using G = WlGeom<NTAP>;
    static_assert(64 * kKMax * 2 + S * G::STAGE + kNW * 4096 <= 160 * 1024, "LDS");
    static_assert(kMaxTiles * G::PW <= 32, "validity bits: kMaxTiles * PW <= 32");
    const WlGrid g = wlds_grid(p, M);
    const int o0 = p.off[0], o1 = p.off[p.ntaps - 1];
    // MTTS_WLDS_DBG (diagnostics only): bit 0 = no MFMAs, bit 1 = no A staging
    static const int dbg = [] { const char *e = getenv("MTTS_WLDS_DBG"); return e ? atoi(e) : 0; }();
    hipLaunchKernelGGL((conv_gemm_wlds_kernel<ABF16, NPL, NTAP, S, EK>), dim3((unsigned)(g.ncg * g.R)), dim3(kNT), 0, st, p,
                       g.ncg, g.mtiles, std::min(o0, o1), dbg);
    return mtts::check_launch("conv_gemm_wlds_kernel");
}

template <bool ABF16, int NPL, int NTAP>
int launch_wlds_t(const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    return mtts::gemm_epilogue_kind(p) == mtts::EK_LIN_C16 ? launch_wlds_e<ABF16, NPL, NTAP, mtts::EK_LIN_C16>(p, M, st)
                                                            : launch_wlds_e<ABF16, NPL, NTAP, mtts::EK_LIN_C32>(p, M, st);
}

template <bool ABF16, int NPL>
int launch_wlds_n(const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    switch (p.ntaps) {
        case 1: return launch_wlds_t<ABF16, NPL, 1>(p, M, st);
        case 2: return launch_wlds_t<ABF16, NPL, 2>(p, M, st);
        default: return launch_wlds_t<ABF16, NPL, 3>(p, M, st);
    }
}

}  // namespace

namespace mtts {

// bf16 MFMA on one or two weight planes; 1..3 taps at stride 1 over whole utterances (Ti == To); K = taps * cin <= 768
// with whole 64-byte channel chunks (cin % 32 bf16 / % 16 fp32); a 0/1 row mask or none; no activation / pre-activation
// (the plain bf16 / fp32 C epilogue kinds, with a bias at most: no residual / c_scale / dropout); 16-byte epilogue
bool conv_gemm_wlds_applies(const mtts_conv_gemm_args &p) {
    if (p.ntaps < 1 || p.ntaps > 3 || p.in_stride != 1 || p.Ti != p.To) return false;
    if (p.ntaps > 1 && p.off[1] - p.off[0] != 1 && p.off[1] - p.off[0] != -1) return false;
    if (p.K != p.ntaps * p.cin || p.K > kKMax || p.K % 128) return false;  // (the W swizzle: 16-chunk groups)
    if (p.flags & (MTTS_GEMM_F_A_SPLIT | MTTS_GEMM_F_SPLIT3)) return false;
    if (p.a_scale && !(p.flags & MTTS_GEMM_F_BINARY_SCALE)) return false;
    const bool a16 = p.flags & MTTS_GEMM_F_A_BF16;
    const int es = a16 ? 2 : 4;
    if (p.cin % (64 / es) || p.lda % (16 / es) || (uintptr_t)p.A % 16 || (uintptr_t)p.W % 16 || p.Kp % 8) return false;
    const int k = gemm_epilogue_kind(p);
    if (k != EK_LIN_C16 && k != EK_LIN_C32) return false;
    // no epilogue stream but the output: a global load inside the DMA pipeline waits for (drains) every DMA in flight
    if (p.residual || p.c_scale || p.dropout_p > 0.f) return false;
    if ((long long)p.nb * p.Ti * p.lda * es >= (1ll << 31) - (1ll << 20)) return false;
    const int npl = (p.flags & MTTS_GEMM_F_W_SPLIT) ? 2 : 1;
    if ((long long)npl * p.N * p.Kp * 2 >= (1ll << 31) - (1ll << 20)) return false;
    return gemm_epilogue_vec_ok(p) && gemm_epilogue_vec8_ok(p);
}

int conv_gemm_wlds_launch(const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    const bool a16 = p.flags & MTTS_GEMM_F_A_BF16, w2 = p.flags & MTTS_GEMM_F_W_SPLIT;
    if (a16) return w2 ? launch_wlds_n<true, 2>(p, M, st) : launch_wlds_n<true, 1>(p, M, st);
    return w2 ? launch_wlds_n<false, 2>(p, M, st) : launch_wlds_n<false, 1>(p, M, st);
}

}  // namespace mtts
