// Weight-resident bf16 implicit GEMM (round 6): the decoder's k = 1 / 2 / 3 convs and linears with K <= 768 --
// Resnet1D's Block1D convs, the transposed conv's phases, their dgrads, the q|k|v dgrad -- behind mtts_conv_gemm
// (include/mtts_decoder.h), schedule id MTTS_GEMM_WLDS.
//
// Why: the LDS-DMA kernels (conv_gemm_glds.hip) stream the packed weights through LDS again for every 64-row tile.
// On the decoder's 256-column convs that is most of what a workgroup loads (W 256 x 768 x 2 B per tile per plane
// against 64 x 768 x 2 B of A), and the per-CU L2 -> LDS fill (~70 GB/s, MI355X_MICROARCH.md 'gather into LDS';
// round-5 fill probe) bounds them.  Here a workgroup owns 64 weight rows -- 64 output columns (one plane) or 32
// columns x two planes (the parity policy's split weights) -- over the whole reduction K <= 768: 96 KiB of LDS,
// loaded ONCE.  Its four waves then walk their own blocks of 32 * TM rows independently (no barrier after the W
// load): A goes straight to registers through a compiler-tracked prefetch ring PD substeps deep (a k = 3 conv reads
// each 16-channel chunk at the three tap offsets back to back, so the shifted rows come from L1), W fragments come
// from LDS, and the next block's first loads are issued during the current block's tail.
//
// History (round 6, tools/r6/gpu_wlds*.sh): a first version staged A through an LDS-DMA ring shared by the four
// waves; the W image leaves only ~50 KiB of LDS for that ring, each step was barrier- and latency-bound at ~0.5-1 us
// whatever it carried (diagnostic switches: 24.8 of 29.7 us without MFMAs and without A staging), and it ran 20-90 %
// slower than the LDS-DMA kernels on every step shape.
//
// Numerics: fp32 accumulation of bf16 products in (64-channel chunk, tap, permuted 16-k substep) order -- not bitwise
// the LDS-DMA kernels' tap-major order; within fp32 accumulation error of them (tests/test_gemm_wlds_gpu.py).
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

constexpr int kNW = 4, kNT = 64 * kNW;
constexpr int kKMax = 768;  // the W image: 64 rows x K bf16
constexpr uint32_t kOob = mtts::kDmaOob;

__device__ float g_wl_zero[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // never written: invalid tap rows

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

// W image row-major, 16-byte chunk c of row w at ((c & ~15) | ((c & 15) ^ (w & 15))): 16 lanes reading one logical
// chunk of 16 consecutive rows hit distinct banks
__device__ __forceinline__ int w_swz(int row, int c) { return ((c & ~15) | ((c & 15) ^ (row & 15))) << 4; }

// One A fragment slot of the prefetch ring: TM row blocks x (bf16: 8 values in one uint4 | fp32: 8 values in two)
template <bool ABF16, int TM>
struct AFrag {
    uint4 v[TM][ABF16 ? 1 : 2];
};

// ABF16: A storage; NPL: weight planes; NTAP taps (stride 1); KS = K / 16 substeps; TM: 32-row blocks per wave block;
// PD: prefetch distance in substeps (PD + 1 divides KS: ring slots are compile-time per substep in every block)
template <bool ABF16, int NPL, int NTAP, int KS, int TM, int PD, int EK>
__global__ __launch_bounds__(kNT, 1) void conv_gemm_wlds_kernel(mtts_conv_gemm_args p, int ncg, int nblk) {
    static_assert(KS % (PD + 1) == 0, "ring slots repeat every block");
    constexpr int ES = ABF16 ? 2 : 4;
    constexpr int K = 16 * KS, CIN = K / NTAP;
    constexpr int TN = NPL == 2 ? 1 : 2;                       // 32-column accumulator blocks per wave
    constexpr int BMW = 32 * TM;                                // rows per wave block
    constexpr int NS = PD + 1;
    static_assert(CIN % 64 == 0 && K <= kKMax, "shape: whole 64-channel chunks per tap");
    __shared__ __attribute__((aligned(1024))) unsigned char sw[64 * K * 2];
    __shared__ __attribute__((aligned(16))) float sepi[kNW * 1024];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lr = lane & 31, lh = lane >> 5;
    const int M = p.nb * p.To;
    const int nwg = gridDim.x, R = nwg / ncg;
    const int g = mtts::xcd_relabel(blockIdx.x, nwg);
    const int cg = g % ncg, r = g / ncg;
    const int n0 = cg * (NPL == 2 ? 32 : 64);
    const int dstep = NTAP > 1 ? p.off[1] - p.off[0] : 0;
    const float inv_to = 1.0f / (float)p.To;

    // ---- W image by LDS-DMA (64 rows x K; row w = plane * 32 + column, or column), then the bias of this lane's
    // accumulator columns (added to the finished accumulators: the epilogue's own bias load would wait, in order,
    // for every prefetch load issued before it)
    {
        const u32x4 rsw = mtts::make_rsrc(p.W, (uint32_t)((long long)NPL * p.N * p.Kp * 2));
        const uint32_t lw = mtts::lds_addr(sw);
        constexpr int CPR = K / 8;  // 16-byte chunks per W row
        for (int q = wave; q < K / 8; q += kNW) {
            const int t = 64 * q + lane, w = t / CPR, pc = t - w * CPR;
            const int c = (pc & ~15) | ((pc & 15) ^ (w & 15));
            const int pl = NPL == 2 ? w >> 5 : 0, n = n0 + (NPL == 2 ? w & 31 : w);
            const uint32_t vw = n < p.N ? (uint32_t)((((long long)pl * p.N + n) * p.Kp + c * 8) * 2) : kOob;
            mtts::bload16(vw, rsw, 0u, __builtin_amdgcn_readfirstlane(lw + q * 1024));
        }
    }
    float bias[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + 32 * j + lr;
        bias[j] = p.bias && n < p.N ? p.bias[n] : 0.f;
    }
    mtts::wait_vmcnt<0>();
    __syncthreads();  // the W image is complete and read-only from here on

    mtts_conv_gemm_args pe = p;
    pe.bias = nullptr;

    // ---- A addressing.  The reduction runs over 64-channel chunks c, tap j inside a chunk, 4 substeps s inside a
    // tap, and a substep's 16 k are NOT 16 consecutive channels: lane half lh takes channels 64 c + 32 lh + 8 s ..
    // + 8 (W's fragments follow the same permutation).  So a lane's 4 substeps read 32 contiguous channels of its
    // row and the 64 lanes of 4 consecutive loads cover whole 128-byte lines: with 16 consecutive channels per
    // substep (the MFMA's natural k order) every load touched 32 lines for 32 bytes each, and with four waves'
    // blocks L1 could not hold the lines until the next chunk came back -- ~4x the bytes from L2.
    // base: the lane's row of block row i at tap j (+ its 32-channel half), ok: 0 when the tap row is invalid
    // (every load of it then reads the zero buffer)
    const unsigned char *abase = reinterpret_cast<const unsigned char *>(p.A);
    const unsigned char *zero = reinterpret_cast<const unsigned char *>(g_wl_zero);
    auto row_ok = [&](int m, int j, int &src) {  // tap j of output row m: in its utterance (and m < M)
        int b = 0, u = 0;
        mtts::divmod_fast(m < M ? m : 0, p.To, inv_to, b, u);
        const int o = p.off[0] + j * dstep;
        src = m + o;
        return m < M && u + o >= 0 && u + o < p.Ti;
    };
    const unsigned char *base[TM][NTAP], *nbase[TM][NTAP];
    int stp[TM][NTAP], nstp[TM][NTAP];  // 1: valid, 0: zero buffer
    float mk[TM][NTAP];
    auto load_masks = [&](int blk) {  // the next block's input-row masks (used NS substeps before it starts)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < NTAP; ++j) {
                int src = 0;
                const bool ok = blk < nblk && row_ok(blk * BMW + 32 * i + lr, j, src);
                mk[i][j] = p.a_scale ? p.a_scale[ok ? src : 0] : 1.f;
            }
    };
    auto set_bases = [&](int blk, const unsigned char *(&bs)[TM][NTAP], int (&sp)[TM][NTAP]) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < NTAP; ++j) {
                int src = 0;
                const bool ok = blk < nblk && row_ok(blk * BMW + 32 * i + lr, j, src) && mk[i][j] != 0.f;
                bs[i][j] = ok ? abase + ((long long)src * p.lda + 32 * lh) * ES : zero;
                sp[i][j] = ok ? 1 : 0;
            }
    };
    // substep t of a block = (chunk t / (4 NTAP), tap (t / 4) % NTAP, s = t % 4): the taps of one chunk back to back
    // (the shifted rows come from L1)
    auto load = [&](const unsigned char *(&bs)[TM][NTAP], int (&sp)[TM][NTAP], int t, AFrag<ABF16, TM> &f) {
        const int c = t / (4 * NTAP), j = (t / 4) % NTAP, sub = t % 4;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const unsigned char *q = bs[i][j] + sp[i][j] * ((64 * c + 8 * sub) * ES);
            f.v[i][0] = *reinterpret_cast<const uint4 *>(q);
            if constexpr (!ABF16) f.v[i][1] = *reinterpret_cast<const uint4 *>(q + 16);
        }
    };

    int blk = r + R * wave;  // this wave's blocks: r + R * (wave + 4 i)
    AFrag<ABF16, TM> ring[NS];
    load_masks(blk);
    set_bases(blk, base, stp);
#pragma unroll
    for (int t = 0; t < PD; ++t) load(base, stp, t, ring[t]);

    const int wrow0 = lr * K * 2, wrow1 = (32 + lr) * K * 2;  // this lane's two W rows (w & 15 == lr & 15)
    for (; blk < nblk; blk += kNW * R) {
        const int nxt = blk + kNW * R;
        load_masks(nxt);  // (always issued: a zero-step base for a missing next block reads the zero buffer)
        f32x16 acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
        // W fragments of substep t (k = j * CIN + 64 c + 32 lh + 8 s, the permutation above), read one substep ahead;
        // a scheduling barrier per substep keeps the compiler from hoisting every read of the unrolled block (it
        // spilled at two planes)
        auto wread = [&](int t, bf16x8 (&b)[2]) {
            const int c = t / (4 * NTAP), j = (t / 4) % NTAP, sub = t % 4;
            const int so = w_swz(lr, (j * CIN + 64 * c + 8 * sub) / 8 + 4 * lh);
            b[0] = *reinterpret_cast<const bf16x8 *>(sw + wrow0 + so);
            b[1] = *reinterpret_cast<const bf16x8 *>(sw + wrow1 + so);
        };
        bf16x8 wb[2][2];
        wread(0, wb[0]);
#pragma unroll
        for (int t = 0; t < KS; ++t) {
            if (t == KS - PD) set_bases(nxt, nbase, nstp);
            if (t + PD < KS) load(base, stp, t + PD, ring[(t + PD) % NS]);
            else load(nbase, nstp, t + PD - KS, ring[(t + PD) % NS]);
            if (t + 1 < KS) wread(t + 1, wb[(t + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            const bf16x8 b0 = wb[t & 1][0], b1 = wb[t & 1][1];
            const AFrag<ABF16, TM> &f = ring[t % NS];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                bf16x8 af;
                if constexpr (ABF16) {
                    af = __builtin_bit_cast(bf16x8, f.v[i][0]);
                } else {
                    const uint4 x0 = f.v[i][0], x1 = f.v[i][1];
                    af = __builtin_bit_cast(
                        bf16x8, make_uint4(pack2(__uint_as_float(x0.x), __uint_as_float(x0.y)),
                                           pack2(__uint_as_float(x0.z), __uint_as_float(x0.w)),
                                           pack2(__uint_as_float(x1.x), __uint_as_float(x1.y)),
                                           pack2(__uint_as_float(x1.z), __uint_as_float(x1.w))));
                }
                if constexpr (NPL == 2) {
                    acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b0, acc[i][0], 0, 0, 0);
                    acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b1, acc[i][0], 0, 0, 0);
                } else {
                    acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b0, acc[i][0], 0, 0, 0);
                    acc[i][TN - 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b1, acc[i][TN - 1], 0, 0, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (p.bias) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int v = 0; v < 16; ++v) acc[i][j][v] += bias[j];
        }
        mtts::gemm_epilogue_vec_v<8, TM, TN, EK, false>(pe, acc, sepi + wave * 1024, blk * BMW, n0, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < NTAP; ++j) {
                base[i][j] = nbase[i][j];
                stp[i][j] = nstp[i][j];
            }
    }
}

struct WlGrid {
    int ncg, nblk, R;
};

WlGrid wlds_grid(const mtts_conv_gemm_args &p, int M, int bmw) {
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
    g.nblk = (M + bmw - 1) / bmw;
    g.R = std::max(1, std::min((g.nblk + kNW - 1) / kNW, cus / g.ncg));
    return g;
}

template <bool ABF16, int NPL, int NTAP, int KS, int EK>
int launch_wlds_e(const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    constexpr int TM = 2;
    constexpr int PD = ABF16 ? 15 : 7;
    const WlGrid g = wlds_grid(p, M, 32 * TM);
    hipLaunchKernelGGL((conv_gemm_wlds_kernel<ABF16, NPL, NTAP, KS, TM, PD, EK>), dim3((unsigned)(g.ncg * g.R)), dim3(kNT),
                       0, st, p, g.ncg, g.nblk);
    return mtts::check_launch("conv_gemm_wlds_kernel");
}

template <bool ABF16, int NPL, int NTAP, int KS>
int launch_wlds_k(const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    switch (mtts::gemm_epilogue_kind(p)) {
        case mtts::EK_LIN_C16: return launch_wlds_e<ABF16, NPL, NTAP, KS, mtts::EK_LIN_C16>(p, M, st);
        case mtts::EK_LIN_C32: return launch_wlds_e<ABF16, NPL, NTAP, KS, mtts::EK_LIN_C32>(p, M, st);
        default: return launch_wlds_e<ABF16, NPL, NTAP, KS, mtts::EK_RT>(p, M, st);
    }
}

// (taps, K) instantiated: (3, 768) the k = 3 convs over 256 channels; (2, 512) the transposed conv's phases; (1, 768)
// the q|k|v dgrad; (1, 512), (1, 256) the other 256 / 512-wide linears
template <bool ABF16, int NPL>
int launch_wlds_n(const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    if (p.ntaps == 3 && p.K == 768) return launch_wlds_k<ABF16, NPL, 3, 48>(p, M, st);
    if (p.ntaps == 2 && p.K == 512) return launch_wlds_k<ABF16, NPL, 2, 32>(p, M, st);
    if constexpr (ABF16) {  // (an fp32 A at K = 768, one tap, spilled; no step launch has it)
        if (p.ntaps == 1 && p.K == 768) return launch_wlds_k<ABF16, NPL, 1, 48>(p, M, st);
    }
    if (p.ntaps == 1 && p.K == 512) return launch_wlds_k<ABF16, NPL, 1, 32>(p, M, st);
    if (p.ntaps == 1 && p.K == 256) return launch_wlds_k<ABF16, NPL, 1, 16>(p, M, st);
    return mtts::fail(MTTS_ERR_UNSUPPORTED, "conv_gemm: weight-resident schedule: (taps, K) not instantiated");
}

}  // namespace

namespace mtts {

// bf16 MFMA on one or two weight planes; (taps, K) in {(3, 768), (2, 512), (1, 768; bf16 A), (1, 512), (1, 256)} at stride 1
// over whole utterances (Ti == To); a 0/1 row mask or none; 16-byte aligned A rows; any epilogue without an
// activation / pre-activation (the 16-byte epilogue: N % 8)
bool conv_gemm_wlds_applies(const mtts_conv_gemm_args &p) {
    if (p.ntaps < 1 || p.ntaps > 3 || p.in_stride != 1 || p.Ti != p.To) return false;
    if (p.ntaps > 1 && p.off[1] - p.off[0] != 1 && p.off[1] - p.off[0] != -1) return false;
    const bool kok = (p.ntaps == 3 && p.K == 768) || (p.ntaps == 2 && p.K == 512) ||
                     (p.ntaps == 1 && (p.K == 768 || p.K == 512 || p.K == 256));
    if (!kok || p.K != p.ntaps * p.cin) return false;
    if (!(p.flags & MTTS_GEMM_F_A_BF16) && p.ntaps == 1 && p.K == 768) return false;  // not instantiated
    if (p.flags & (MTTS_GEMM_F_A_SPLIT | MTTS_GEMM_F_SPLIT3)) return false;
    if (p.a_scale && !(p.flags & MTTS_GEMM_F_BINARY_SCALE)) return false;
    const bool a16 = p.flags & MTTS_GEMM_F_A_BF16;
    const int es = a16 ? 2 : 4;
    if (p.lda % (16 / es) || (uintptr_t)p.A % 16 || (uintptr_t)p.W % 16 || p.Kp % 8) return false;
    if (p.act != MTTS_ACT_NONE || p.C_pre) return false;
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
