// bf16 implicit GEMM with LDS-DMA staging (global_load_lds_dwordx4) of both operands -- the default
// bf16 schedule of mtts_conv_gemm for the decoder / encoder convs and linears.
//
// Same contract as conv_gemm_kernel (include/mtts_decoder.h), for precision MTTS_PREC_BF16 with
// a_scale either NULL or a 0/1 row mask (MTTS_GEMM_F_BINARY_SCALE).  Why a second kernel: the
// register-staged kernel spends ~45 VALU instructions per MFMA on staging (fp32 loads, row-mask
// multiply, bf16 conversion, validity selects, LDS stores; SQ_INSTS_VALU / SQ_INSTS_MFMA on the step's
// 19200 x 256 x 768 conv) and is issue-bound at ~9 % of MFMA peak.  Here the operands go
// HBM/L2 -> LDS with no VGPR round trip:
//   A (fp32 activations): each lane DMAs one 16-byte chunk (4 channels) of one tap row; a row that
//     lies outside [0, Ti) or whose mask is 0 is read from a 16-byte zero constant instead, so the
//     masked / zero-padded operand is formed by address selection alone.  The fp32 -> bf16 conversion
//     moves to the fragment read (4 v_cvt_pk_bf16_f32 per 8 elements).
//   W (packed bf16 [N][Kp]): DMA'd as is.
// LDS images are XOR-swizzled through the per-lane SOURCE address (an LDS-DMA wave instruction fills
// 1 KiB lane-linearly): A rows are 256 B (64 fp32 of one K step), 16-byte chunk c of row r sits at
// c ^ (r & 15); W rows are 128 B, chunk c of row n at c ^ ((n >> 1) & 7).  Both make the MFMA
// fragment reads (ds_read_b128, 16-lane groups) bank-conflict free.
// Pipeline: STAGES LDS buffers, K step 64, loads for step kt + STAGES - 1 issued right after the
// barrier that retires step kt - 1's reads; a counted s_waitcnt vmcnt (never 0 inside the loop) and a
// raw s_barrier (no fence: __syncthreads() would drain the in-flight DMAs) order each buffer.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <utility>

#include "gemm_epilogue.h"
#include "lds_dma.h"
#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
using mtts::f32x16;

__device__ uint4 g_zero16 = {0u, 0u, 0u, 0u};  // never written: source of every masked / out-of-range chunk

// -DMTTS_GEMM_TIMELINE=1 (diagnostic builds only, tools/r6/glds_timeline.py): lane 0 of every wave stamps the
// 100 MHz wall clock into g_tlg ([wave][kTlSlots]: HW ids, start, prologue issued, then per K step: data landed +
// barrier passed / MFMAs issued, loop end, epilogue end); read back by mtts_glds_timeline_read.
#ifndef MTTS_GEMM_TIMELINE
#define MTTS_GEMM_TIMELINE 0
#endif
#if MTTS_GEMM_TIMELINE
constexpr int kTlSlots = 128, kTlWaves = 16384, kTlSteps = 60;
__device__ long long g_tlg[kTlWaves * kTlSlots];
#define MTTS_TLG(slot)                                                                                   \
    do {                                                                                                 \
        const int tl_w = (int)blockIdx.x * NW + wave;                                                    \
        if (lane == 0 && tl_w < kTlWaves && (slot) < kTlSlots) g_tlg[tl_w * kTlSlots + (slot)] = wall_clock64(); \
    } while (0)
#else
#define MTTS_TLG(slot) \
    do {               \
    } while (0)
#endif

constexpr int kBK = 64;

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

using mtts::bload16;
using mtts::glds16;
using mtts::make_rsrc;
using mtts::u32x4;
using mtts::wait_vmcnt;
constexpr uint32_t MTTS_GLDS_OOB = mtts::kDmaOob;

template <int WM, int WN, int TM, int TN, int STAGES, bool ABF16 = false, int NPL = 1>
struct GldsGeom {
    static constexpr int NT = 64 * WM * WN;
    static constexpr int BM = 32 * WM * TM, BN = 32 * WN * TN;
    static constexpr int A_BYTES = BM * kBK * (ABF16 ? 2 : 4);  // fp32 rows of 256 B / bf16 rows of 128 B
    static constexpr int W_BYTES = NPL * BN * kBK * 2;  // bf16 rows of 128 B (NPL weight planes: BN rows each)
    static constexpr int GA = A_BYTES / (NT * 16);  // DMA instructions per thread per K step
    static constexpr int GW = W_BYTES / (NT * 16);
    static_assert(A_BYTES % (NT * 16) == 0 && W_BYTES % (NT * 16) == 0, "tile / threads mismatch");
};

// ABF16: A is bf16 in HBM (MTTS_GEMM_F_A_BF16): 128-byte rows, the same image and swizzle as W, and
// the fragment read needs no conversion.
// LEAN (cin % 64 == 0, so every K step lies inside one tap and K % 64 == 0; 32-bit byte offsets): the
// operands are read through buffer descriptors, the K step advance is a scalar offset and only a tap
// change touches per-lane state -- the register-addressed loop spent ~12 vector instructions per DMA
// on pointer and tap bookkeeping (~26 VALU per MFMA on the 19200 x 256 x 768 conv, SQ counters).
// WS (MTTS_GEMM_F_W_SPLIT): the W image holds BN hi rows then BN lo rows (the lo plane starts N*Kp
// elements after W); each fragment pair issues A*hi and A*lo.
// X3 (MTTS_GEMM_F_SPLIT3, fp32 A, round 4): bf16x6 -- W holds three planes hi / mid / lo (hi + mid + lo = w
// exactly, packed by mtts_pack_weights), the fp32 A fragment is split the same way at the fragment read, and
// every product is the six terms of combined order <= 2^-16 (hi*hi, hi*mid, mid*hi, hi*lo, lo*hi, mid*mid),
// smallest first, into the fp32 accumulator: ~2^-24 relative per product, fp32-faithful (the parity policy's
// text encoder forward at bf16 MFMA rates)
template <int WM, int WN, int TM, int TN, int STAGES, bool ABF16, bool LEAN, bool WS = false, bool X3 = false>
__global__ __launch_bounds__(64 * WM * WN) void conv_gemm_glds_kernel(mtts_conv_gemm_args p, int ksteps, float *part) {
    static_assert(!X3 || (!ABF16 && !WS), "bf16x6: fp32 A, three weight planes");
    constexpr int NPL = X3 ? 3 : (WS ? 2 : 1);
    using G = GldsGeom<WM, WN, TM, TN, STAGES, ABF16, NPL>;
    constexpr int ES = ABF16 ? 2 : 4;        // bytes per A element
    constexpr int RPI = ABF16 ? 8 : 4;       // A rows per 1 KiB DMA instruction
    constexpr int CPR = ABF16 ? 8 : 16;      // 16-byte chunks per A row of one K step
    constexpr int EPC = 16 / ES;             // A elements per chunk
    constexpr int NT = G::NT, BM = G::BM, BN = G::BN, GA = G::GA, GW = G::GW, NW = NT / 64;
    // one __shared__ object per stage and operand, and a K loop unrolled by STAGES so every access
    // names its buffer statically: hipcc then sees that a DMA into one buffer cannot alias the
    // ds_reads of another and does not insert vmcnt(0) before them (one shared array with a runtime
    // stage offset gets a full drain of the in-flight DMAs before every fragment read)
    __shared__ __attribute__((aligned(1024))) unsigned char sA0[G::A_BYTES], sW0[G::W_BYTES];
    __shared__ __attribute__((aligned(1024))) unsigned char sA1[G::A_BYTES], sW1[G::W_BYTES];
    __shared__ __attribute__((aligned(1024))) unsigned char sA2[STAGES > 2 ? G::A_BYTES : 16],
        sW2[STAGES > 2 ? G::W_BYTES : 16];
    auto abuf = [&](auto S) -> unsigned char * {
        if constexpr (decltype(S)::value == 0) return sA0;
        else if constexpr (decltype(S)::value == 1) return sA1;
        else return sA2;
    };
    auto wbuf = [&](auto S) -> unsigned char * {
        if constexpr (decltype(S)::value == 0) return sW0;
        else if constexpr (decltype(S)::value == 1) return sW1;
        else return sW2;
    };
    // LDS byte addresses of the stage buffers, cast from the __shared__ objects themselves (a constant:
    // no generic-pointer null check)
    typedef __attribute__((address_space(3))) unsigned char lds_u8;
    auto lds_addr = [](const lds_u8 *q) { return (uint32_t)(uintptr_t)q; };
    auto abuf_l = [&](auto S) -> uint32_t {
        if constexpr (decltype(S)::value == 0) return lds_addr((const lds_u8 *)sA0);
        else if constexpr (decltype(S)::value == 1) return lds_addr((const lds_u8 *)sA1);
        else return lds_addr((const lds_u8 *)sA2);
    };
    auto wbuf_l = [&](auto S) -> uint32_t {
        if constexpr (decltype(S)::value == 0) return lds_addr((const lds_u8 *)sW0);
        else if constexpr (decltype(S)::value == 1) return lds_addr((const lds_u8 *)sW1);
        else return lds_addr((const lds_u8 *)sW2);
    };

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave / WN, wc = wave % WN;
    const int lr = lane & 31, lh = lane >> 5;
    const int M = p.nb * p.To;
    // split-K (part != NULL): grid = tiles x S, the S splits of a tile adjacent (same XCD); split s
    // reduces K steps [s*ksteps, min(nk, (s+1)*ksteps)) and stores raw fp32 partials to part[s][M][N]
    int m0, n0, kstep0 = 0, nk = (p.K + kBK - 1) / kBK;
    {
        const int nt = (p.N + BN - 1) / BN;
        const int ntiles = ((M + BM - 1) / BM) * nt;
        const int S = gridDim.x / ntiles;
        int t = mtts::xcd_relabel(blockIdx.x, gridDim.x);
        if (S > 1) {
            const int tile = t / S, split = t - tile * S;
            t = tile;
            kstep0 = split * ksteps;
            nk = min(ksteps, nk - kstep0);
        }
        const int mt = t / nt;
        m0 = mt * BM;
        n0 = (t - mt * nt) * BN;
    }
    const float inv_to = 1.0f / (float)p.To;
    const int off0 = p.off[0], offstep = p.ntaps > 1 ? p.off[1] - p.off[0] : 0;

    // ---- A chunk state: DMA instruction i of this wave covers tile rows 4q..4q+3 (q = i*NW + wave);
    // lane -> row 4q + lane/16, LDS slot lane%16 <- logical chunk (lane%16) ^ (row & 15)
    const float *zero = reinterpret_cast<const float *>(&g_zero16);
    const long long tap_delta = ((long long)offstep * p.lda - p.cin) * ES;  // source bytes when a chunk changes tap
    const char *a_src[GA];   // the lane's chunk in the current step (valid when its tap's bit is set)
    int a_ch[GA], a_j[GA];   // channel of the lane's chunk within its tap, and the tap
    uint32_t a_ok[GA];       // bit j: tap j's source row exists and is unmasked
#pragma unroll
    for (int i = 0; i < GA; ++i) {
        const int r = RPI * (i * NW + wave) + lane / CPR;
        const int lc = (lane % CPR) ^ (ABF16 ? ((r >> 1) & 7) : (r & 15));
        const int m = m0 + r;
        int b = 0, u = 0;
        const bool mv = m < M;
        mtts::divmod_fast(mv ? m : 0, p.To, inv_to, b, u);
        uint32_t ok = 0;
        for (int j = 0; j < p.ntaps; ++j) {
            const int irow = u * p.in_stride + off0 + j * offstep;
            bool v = mv && irow >= 0 && irow < p.Ti;
            if (v && p.a_scale) v = p.a_scale[(size_t)b * p.Ti + irow] != 0.f;
            ok |= (uint32_t)v << j;
        }
        a_ok[i] = ok;
        const int k = kstep0 * kBK + lc * EPC;  // the lane's element within the first K step
        a_j[i] = k / p.cin;
        a_ch[i] = k - a_j[i] * p.cin;
        a_src[i] = reinterpret_cast<const char *>(p.A) +
                   ((long long)(b * p.Ti + u * p.in_stride + off0 + a_j[i] * offstep) * p.lda + a_ch[i]) * ES;
    }
    // ---- W chunk state: instruction i covers W rows 8q..8q+7; lane -> row 8q + lane/8, LDS slot lane%8
    // <- logical chunk (lane%8) ^ ((row >> 1) & 7)
    const uint16_t *w_ptr[GW];
    int w_k[GW];
    bool w_nok[GW];
    const size_t w_plane = (size_t)p.N * p.Kp;  // WS / X3: elements from one weight plane to the next
#pragma unroll
    for (int i = 0; i < GW; ++i) {
        const int ni = 8 * (i * NW + wave) + (lane >> 3);  // row of the W image
        const int pl = NPL > 1 ? ni / BN : 0;
        const int n = ni - pl * BN;
        const int lc = (lane & 7) ^ ((ni >> 1) & 7);  // BN % 16 == 0: the lo rows swizzle like the hi rows
        w_nok[i] = n0 + n < p.N;
        w_k[i] = kstep0 * kBK + lc * 8;
        w_ptr[i] = static_cast<const uint16_t *>(p.W) + pl * w_plane + (size_t)(w_nok[i] ? n0 + n : 0) * p.Kp + w_k[i];
    }

    // ---- LEAN state: per chunk the tap-0 element index of its row and the byte offset of the current
    // tap (MTTS_GLDS_OOB when that tap's row is absent or masked); scalar tap / channel-block counters
    const int tapstride = offstep * p.lda;
    int l_row[LEAN ? GA : 1];
    uint32_t l_vo[LEAN ? GA : 1], l_vw[LEAN ? GW : 1];
    int l_tap = 0, l_chs = 0;
    uint32_t l_soa = 0, l_sow = 0;
    u32x4 l_rsa, l_rsw;
    if constexpr (LEAN) {
        const int k0 = kstep0 * kBK;
        l_tap = __builtin_amdgcn_readfirstlane(k0 / p.cin);
        const int ch0 = k0 - l_tap * p.cin;
        l_chs = __builtin_amdgcn_readfirstlane((p.cin - ch0) / kBK);
        l_soa = __builtin_amdgcn_readfirstlane((uint32_t)(ch0 * ES));
        l_sow = __builtin_amdgcn_readfirstlane((uint32_t)(k0 * 2));
        l_rsa = make_rsrc(p.A, (uint32_t)((long long)p.nb * p.Ti * p.lda * ES));
        l_rsw = make_rsrc(p.W, (uint32_t)((long long)NPL * p.N * p.Kp * 2));
#pragma unroll
        for (int i = 0; i < GA; ++i) {
            const int r = RPI * (i * NW + wave) + lane / CPR;
            const int lc = (lane % CPR) ^ (ABF16 ? ((r >> 1) & 7) : (r & 15));
            int b = 0, u = 0;
            mtts::divmod_fast(m0 + r < M ? m0 + r : 0, p.To, inv_to, b, u);
            l_row[i] = (b * p.Ti + u * p.in_stride + off0) * p.lda + lc * EPC;
            l_vo[i] = ((a_ok[i] >> min(l_tap, 31)) & 1u) ? (uint32_t)((l_row[i] + l_tap * tapstride) * ES) : MTTS_GLDS_OOB;
        }
#pragma unroll
        for (int i = 0; i < GW; ++i) {
            const int ni = 8 * (i * NW + wave) + (lane >> 3);
            const int pl = NPL > 1 ? ni / BN : 0;
            const int n = ni - pl * BN;
            const int lc = (lane & 7) ^ ((ni >> 1) & 7);
            l_vw[i] = w_nok[i] ? (uint32_t)((pl * w_plane + (size_t)(n0 + n) * p.Kp + lc * 8) * 2) : MTTS_GLDS_OOB;
        }
    }

    auto issue = [&](auto S) {
        unsigned char *abase = abuf(S);
        unsigned char *wbase = wbuf(S);
        if constexpr (LEAN) {
            const uint32_t la = abuf_l(S), lw = wbuf_l(S);
#pragma unroll
            for (int i = 0; i < GA; ++i)
                bload16(l_vo[i], l_rsa, l_soa, __builtin_amdgcn_readfirstlane(la + (i * NW + wave) * 1024));
#pragma unroll
            for (int i = 0; i < GW; ++i)
                bload16(l_vw[i], l_rsw, l_sow, __builtin_amdgcn_readfirstlane(lw + (i * NW + wave) * 1024));
            l_sow += kBK * 2;
            l_soa += kBK * ES;
            if (--l_chs == 0) {  // next tap (wave-uniform branch; nothing in flight depends on registers)
                ++l_tap;
                l_chs = p.cin / kBK;
                l_soa = 0;
#pragma unroll
                for (int i = 0; i < GA; ++i)
                    l_vo[i] = ((a_ok[i] >> min(l_tap, 31)) & 1u) ? (uint32_t)((l_row[i] + l_tap * tapstride) * ES)
                                                                 : MTTS_GLDS_OOB;
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < GA; ++i) {
            const bool ok = (a_ok[i] >> min(a_j[i], 31)) & 1u;  // a_j >= ntaps (past K): bit is 0
            glds16(ok ? static_cast<const void *>(a_src[i]) : static_cast<const void *>(zero),
                   abase + (i * NW + wave) * 1024);
            a_ch[i] += kBK;
            a_src[i] += kBK * ES;
            const bool w = a_ch[i] >= p.cin;  // cin >= 64: at most one tap change per step
            a_ch[i] -= w ? p.cin : 0;
            a_j[i] += w;
            a_src[i] += w ? tap_delta : 0;
        }
#pragma unroll
        for (int i = 0; i < GW; ++i) {
            const bool ok = w_nok[i] && w_k[i] < p.Kp;
            glds16(ok ? static_cast<const void *>(w_ptr[i]) : static_cast<const void *>(zero),
                   wbase + (i * NW + wave) * 1024);
            w_ptr[i] += kBK;
            w_k[i] += kBK;
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

    auto compute = [&](auto S) {
        const unsigned char *abase = abuf(S);
        const unsigned char *wbase = wbuf(S);
        if constexpr (X3) {
#pragma unroll
            for (int ks = 0; ks < kBK / 16; ++ks) {
                bf16x8 ah[TM], am[TM], al[TM], bh[TN], bm[TN], bl[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int r = wr * 32 * TM + i * 32 + lr;
                    const int c = 4 * ks + 2 * lh;
                    const float4 x0 = *reinterpret_cast<const float4 *>(abase + r * 256 + ((c ^ (r & 15)) << 4));
                    const float4 x1 = *reinterpret_cast<const float4 *>(abase + r * 256 + (((c + 1) ^ (r & 15)) << 4));
                    float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                    uint32_t wh[4], wm[4], wl[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {  // every residual is exact in fp32
                        wh[q] = pack2(v[2 * q], v[2 * q + 1]);
                        v[2 * q] -= __uint_as_float(wh[q] << 16);
                        v[2 * q + 1] -= __uint_as_float(wh[q] & 0xffff0000u);
                        wm[q] = pack2(v[2 * q], v[2 * q + 1]);
                        v[2 * q] -= __uint_as_float(wm[q] << 16);
                        v[2 * q + 1] -= __uint_as_float(wm[q] & 0xffff0000u);
                        wl[q] = pack2(v[2 * q], v[2 * q + 1]);
                    }
                    ah[i] = __builtin_bit_cast(bf16x8, make_uint4(wh[0], wh[1], wh[2], wh[3]));
                    am[i] = __builtin_bit_cast(bf16x8, make_uint4(wm[0], wm[1], wm[2], wm[3]));
                    al[i] = __builtin_bit_cast(bf16x8, make_uint4(wl[0], wl[1], wl[2], wl[3]));
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = wc * 32 * TN + j * 32 + lr;
                    const int c = 2 * ks + lh;
                    const int sw = (c ^ ((n >> 1) & 7)) << 4;  // BN % 16 == 0: every plane swizzles alike
                    bh[j] = *reinterpret_cast<const bf16x8 *>(wbase + n * 128 + sw);
                    bm[j] = *reinterpret_cast<const bf16x8 *>(wbase + (n + BN) * 128 + sw);
                    bl[j] = *reinterpret_cast<const bf16x8 *>(wbase + (n + 2 * BN) * 128 + sw);
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                    }
            }
            return;
        }
#pragma unroll
        for (int ks = 0; ks < kBK / 16; ++ks) {
            bf16x8 af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int r = wr * 32 * TM + i * 32 + lr;
                if constexpr (ABF16) {
                    const int c = 2 * ks + lh;
                    af[i] = *reinterpret_cast<const bf16x8 *>(abase + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
                } else {
                    const int c = 4 * ks + 2 * lh;
                    const float4 x0 = *reinterpret_cast<const float4 *>(abase + r * 256 + ((c ^ (r & 15)) << 4));
                    const float4 x1 =
                        *reinterpret_cast<const float4 *>(abase + r * 256 + (((c + 1) ^ (r & 15)) << 4));
                    const uint4 w =
                        make_uint4(pack2(x0.x, x0.y), pack2(x0.z, x0.w), pack2(x1.x, x1.y), pack2(x1.z, x1.w));
                    af[i] = __builtin_bit_cast(bf16x8, w);
                }
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = wc * 32 * TN + j * 32 + lr;
                const int c = 2 * ks + lh;
                bfr[j] = *reinterpret_cast<const bf16x8 *>(wbase + n * 128 + ((c ^ ((n >> 1) & 7)) << 4));
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            if constexpr (WS) {
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = BN + wc * 32 * TN + j * 32 + lr;
                    const int c = 2 * ks + lh;
                    bfr[j] = *reinterpret_cast<const bf16x8 *>(wbase + n * 128 + ((c ^ ((n >> 1) & 7)) << 4));
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        }
    };

#if MTTS_GEMM_TIMELINE
    if (lane == 0 && (int)blockIdx.x * NW + wave < kTlWaves)
        g_tlg[((int)blockIdx.x * NW + wave) * kTlSlots] =
            ((long long)__smid() << 32) | (long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    MTTS_TLG(1);
#endif
    // prologue: steps 0 .. STAGES-2 in flight (steps past nk DMA zeros into their buffer: harmless)
    issue(std::integral_constant<int, 0>{});
    if constexpr (STAGES > 2) issue(std::integral_constant<int, 1>{});
    MTTS_TLG(2);
    // step kt uses buffer kt % STAGES and refills buffer (kt + STAGES - 1) % STAGES, which step kt-1 read
    int tl_k = 0;
    (void)tl_k;
    auto step = [&](auto S) {
        constexpr int cur = decltype(S)::value, nxt = (cur + STAGES - 1) % STAGES;
        wait_vmcnt<(GA + GW) * (STAGES - 2)>();  // this wave's DMAs for step kt have landed
        mtts::lds_barrier();                       // ... everyone's, and step kt-1's reads are done
#if MTTS_GEMM_TIMELINE
        if (tl_k < kTlSteps) MTTS_TLG(3 + 2 * tl_k);
#endif
        issue(std::integral_constant<int, nxt>{});
        compute(S);
#if MTTS_GEMM_TIMELINE
        __builtin_amdgcn_sched_barrier(0);
        if (tl_k < kTlSteps) MTTS_TLG(4 + 2 * tl_k);
        ++tl_k;
#endif
    };
    for (int kt = 0; kt < nk; kt += STAGES) {
        step(std::integral_constant<int, 0>{});
        if (kt + 1 >= nk) break;
        step(std::integral_constant<int, 1>{});
        if constexpr (STAGES > 2) {
            if (kt + 2 >= nk) break;
            step(std::integral_constant<int, 2>{});
        }
    }
    wait_vmcnt<0>();  // no DMA may still target this workgroup's LDS when it retires
    MTTS_TLG(kTlSlots - 2);
    if (part || mtts::gemm_epilogue_vec_ok(p)) {
        mtts::lds_barrier();  // every wave is past its last fragment read: the buffers are free
        unsigned char *stage = wave % 4 == 0 ? sA0 : wave % 4 == 1 ? sW0 : wave % 4 == 2 ? sA1 : sW1;
        float *st = reinterpret_cast<float *>(stage + (wave / 4) * 4096);
        if (part)
            mtts::gemm_store_partial<TM, TN>(p, acc, st, part + (size_t)(kstep0 / ksteps) * M * p.N,
                                             m0 + wr * 32 * TM, n0 + wc * 32 * TN, lane);
        else
            mtts::gemm_epilogue_vec<TM, TN>(p, acc, st, m0 + wr * 32 * TM, n0 + wc * 32 * TN, lane);
    } else {
        mtts::gemm_epilogue<TM, TN>(p, acc, m0 + wr * 32 * TM, n0 + wc * 32 * TN, lr, lh);
    }
    MTTS_TLG(kTlSlots - 1);
}

// Split-K combine: out = epilogue(sum_s part[s][m][n..n+3]) summed in split order (deterministic).
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(mtts_conv_gemm_args p, const float *__restrict__ part,
                                                              int S) {
    const int M = p.nb * p.To, n4 = p.N >> 2;
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)M * n4) return;
    const int m = (int)(idx / n4), n = (int)(idx - (long long)m * n4) * 4;
    const size_t slab = (size_t)M * p.N;
    float4 a = *reinterpret_cast<const float4 *>(part + (size_t)m * p.N + n);
    for (int s = 1; s < S; ++s) {
        const float4 b = *reinterpret_cast<const float4 *>(part + s * slab + (size_t)m * p.N + n);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float4 bn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.bias) bn = *reinterpret_cast<const float4 *>(p.bias + n);
    float e[4] = {a.x + bn.x, a.y + bn.y, a.z + bn.z, a.w + bn.w};
    int b, u;
    mtts::divmod_fast(m, p.To, 1.0f / (float)p.To, b, u);
    uint32_t s0 = 0, s1 = 0;
    float keep = 1.f;
    if (p.dropout_p > 0.f) {
        s0 = p.seed[0];
        s1 = p.seed[1];
        keep = mtts::dropout_scale(p.dropout_p);
    }
    mtts::epilogue_row4(p, b * p.To_full + u * p.out_stride + p.out_off, n, e, s0, s1, keep);
}

struct GldsCfg {
    int wm, wn, tm, tn, stages;
    bool f32a, bf16a;  // which A storages have an instantiation (LDS <= 160 KiB, registers)
};
constexpr GldsCfg kGlds[] = {
    {1, 4, 2, 2, 2, true, false},   // 32: 64 x 256, 256 thr, 2 stages (96 KiB)
    {1, 4, 2, 2, 3, false, false},  // 33: 64 x 256, 3 stages (144 KiB; fp32 A spills: 7x slower)
    {2, 2, 2, 2, 2, true, false},   // 34: 128 x 128, 2 stages (96 KiB)
    {2, 2, 2, 2, 3, false, false},  // 35: 128 x 128, 3 stages (144 KiB; fp32 A spills: 7x slower)
    {1, 4, 1, 2, 2, true, false},   // 36: 32 x 256, 2 stages (80 KiB)
    {1, 4, 1, 2, 3, true, false},   // 37: 32 x 256, 3 stages (120 KiB)
    {2, 2, 1, 2, 2, true, false},   // 38: 64 x 128, 2 stages (64 KiB)
    {2, 2, 1, 2, 3, true, false},   // 39: 64 x 128, 3 stages (96 KiB)
    {1, 4, 1, 1, 3, true, false},   // 40: 32 x 128, 3 stages (72 KiB)
    {2, 4, 1, 2, 2, true, true},    // 41: 64 x 256, 512 thr (waves 32 x 64), 2 stages (96 KiB)
    {2, 4, 1, 2, 3, true, true},    // 42: 64 x 256, 512 thr, 3 stages (144 KiB)
    {1, 2, 2, 2, 3, true, false},   // 43: 64 x 128, 128 thr (waves 64 x 64), 3 stages (96 KiB)
    {2, 2, 1, 1, 3, true, true},    // 44: 64 x 64, 3 stages (72 KiB)
    {2, 2, 1, 1, 2, true, false},   // 45: 64 x 64, 2 stages (48 KiB)
    {2, 4, 2, 2, 2, true, true},    // 46: 128 x 256, 512 thr (waves 64 x 64), 2 stages (128 KiB)
    {4, 2, 1, 2, 2, true, false},   // 47: 128 x 128, 512 thr (waves 32 x 64), 2 stages (96 KiB)
};
constexpr int kNumGlds = sizeof(kGlds) / sizeof(kGlds[0]);

}  // namespace

namespace mtts {
// The LEAN loop needs whole-tap K steps and 32-bit byte offsets with room for MTTS_GLDS_OOB.
bool conv_gemm_glds_lean(const mtts_conv_gemm_args &p) {
    static const bool off = [] {
        const char *e = getenv("MTTS_GLDS_LEAN");
        return e && e[0] == '0';
    }();
    const int es = (p.flags & MTTS_GEMM_F_A_BF16) ? 2 : 4;
    return !off && p.cin % kBK == 0 && (long long)p.nb * p.Ti * p.lda * es < (1ll << 31) &&
           (long long)p.N * p.Kp * 2 < (1ll << 31);
}
}  // namespace mtts

namespace {

template <int C, bool ABF16, bool WS = false, bool X3 = false>
int launch_glds_t(const mtts_conv_gemm_args &p, int M, int splits, float *part, hipStream_t st) {
    constexpr GldsCfg c = kGlds[C];
    using G = GldsGeom<c.wm, c.wn, c.tm, c.tn, c.stages, ABF16, X3 ? 3 : (WS ? 2 : 1)>;
    static_assert((!WS && !X3) || c.stages * (G::A_BYTES + G::W_BYTES) <= 160 * 1024, "split-weight stages fit LDS");
    auto kern = mtts::conv_gemm_glds_lean(p) ? conv_gemm_glds_kernel<c.wm, c.wn, c.tm, c.tn, c.stages, ABF16, true, WS, X3>
                                : conv_gemm_glds_kernel<c.wm, c.wn, c.tm, c.tn, c.stages, ABF16, false, WS, X3>;
    const int nk = (p.K + kBK - 1) / kBK;
    const int ksteps = (nk + splits - 1) / splits;
    const int S = splits > 1 ? (nk + ksteps - 1) / ksteps : 1;  // every split non-empty
    dim3 grid((unsigned)(((M + G::BM - 1) / G::BM) * ((p.N + G::BN - 1) / G::BN) * S));
    hipLaunchKernelGGL(kern, grid, dim3(G::NT), 0, st, p, ksteps, S > 1 ? part : nullptr);
    int rc = mtts::check_launch("conv_gemm_glds");
    if (rc || S == 1) return rc;
    const long long n4 = (long long)M * (p.N / 4);
    hipLaunchKernelGGL(splitk_epilogue_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, p,
                       (const float *)part, S);
    return mtts::check_launch("splitk_epilogue_kernel");
}

// Split-weight operands (MTTS_GEMM_F_W_SPLIT) run three instantiations: 64 x 64 three-stage (44) or
// two-stage (45), and 64 x 256 two-stage (41, 144 KiB with bf16 A, 160 KiB with fp32 A) for the wide tiles
// (a 128 x 128 two-stage split-weight instance, round 4, ran 3-5x slower than the 64-row ones on the FFN
// up-projection -- tools/r4/ff1_probe.py, profiles/r04/sweeps/ff1_probe.txt -- and was removed)
template <int C>
int launch_glds_ws(const mtts_conv_gemm_args &p, int M, int splits, float *part, hipStream_t st) {
    constexpr int W = kGlds[C].wn * kGlds[C].tn * 32 >= 128 ? 9 : (kGlds[C].stages == 2 ? 13 : 12);
    if (p.flags & MTTS_GEMM_F_A_BF16) {
        if constexpr (kGlds[W].bf16a) return launch_glds_t<W, true, true>(p, M, splits, part, st);
        else return launch_glds_t<9, true, true>(p, M, splits, part, st);
    }
    return launch_glds_t<W, false, true>(p, M, splits, part, st);
}

// bf16x6 (MTTS_GEMM_F_SPLIT3, fp32 A): 64 x 64 tiles, three stages (44: 120 KiB) or two (45)
template <int C>
int launch_glds_x3(const mtts_conv_gemm_args &p, int M, int splits, float *part, hipStream_t st) {
    if constexpr (kGlds[C].stages >= 3) return launch_glds_t<12, false, false, true>(p, M, splits, part, st);
    else return launch_glds_t<13, false, false, true>(p, M, splits, part, st);
}

// A schedule without an instantiation for the operand's storage runs the 64 x 256 two-stage one (41)
template <int C>
int launch_glds(const mtts_conv_gemm_args &p, int M, int splits, float *part, hipStream_t st) {
    if (p.flags & MTTS_GEMM_F_SPLIT3) return launch_glds_x3<C>(p, M, splits, part, st);
    if (p.flags & MTTS_GEMM_F_W_SPLIT) return launch_glds_ws<C>(p, M, splits, part, st);
    if (p.flags & MTTS_GEMM_F_A_BF16) {
        if constexpr (kGlds[C].bf16a) return launch_glds_t<C, true>(p, M, splits, part, st);
        else return launch_glds_t<9, true>(p, M, splits, part, st);
    }
    if constexpr (kGlds[C].f32a) return launch_glds_t<C, false>(p, M, splits, part, st);
    else return launch_glds_t<9, false>(p, M, splits, part, st);
}

template <int... I>
int launch_glds_id(int id, const mtts_conv_gemm_args &p, int M, int splits, float *part, hipStream_t st,
                   std::integer_sequence<int, I...>) {
    int rc = MTTS_ERR_INVALID_ARG;
    ((id == I ? (rc = launch_glds<I>(p, M, splits, part, st), true) : false) || ...);
    return rc;
}

}  // namespace

namespace mtts {

int conv_gemm_glds_num_cfgs() { return kNumGlds; }

// Whether the LDS-DMA kernels can run this GEMM (bf16; 16-byte aligned rows; 0/1 row mask or none;
// 32-bit element offsets).
bool conv_gemm_glds_applies(const mtts_conv_gemm_args &p) {
    if (p.a_scale && !(p.flags & MTTS_GEMM_F_BINARY_SCALE)) return false;
    if (p.cin < kBK || p.cin % 4 || p.lda % 4 || p.Kp % 8) return false;
    if ((p.flags & MTTS_GEMM_F_A_BF16) && (p.cin % 8 || p.lda % 8 || (uintptr_t)p.A % 16)) return false;
    const long long arows = (long long)p.nb * p.Ti;
    if (arows * p.lda >= (1ll << 31) - (1ll << 20)) return false;
    return true;
}

size_t conv_gemm_glds_splitk_bytes(const mtts_conv_gemm_args &p, int splits) {
    if (splits <= 1) return 0;
    const int nk = (p.K + kBK - 1) / kBK;
    const int ksteps = (nk + splits - 1) / splits;
    const int S = (nk + ksteps - 1) / ksteps;
    return S > 1 ? (size_t)S * p.nb * p.To * p.N * sizeof(float) : 0;
}

int splitk_combine(const mtts_conv_gemm_args &p, int M, const float *part, int S, hipStream_t st) {
    const long long n4 = (long long)M * (p.N / 4);
    hipLaunchKernelGGL(splitk_epilogue_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, p, part, S);
    return mtts::check_launch("splitk_epilogue_kernel");
}

int conv_gemm_glds_launch(int id, const mtts_conv_gemm_args &p, int M, int splits, float *part, hipStream_t st) {
    return launch_glds_id(id, p, M, splits, part, st, std::make_integer_sequence<int, kNumGlds>{});
}
}  // namespace mtts

#if MTTS_GEMM_TIMELINE
// diagnostic builds: copy (or zero, host == NULL) the LDS-DMA kernels' timeline buffer; returns its size in bytes
extern "C" long long mtts_glds_timeline_read(void *host) {
    const size_t bytes = sizeof(long long) * kTlWaves * kTlSlots;
    if (host) {
        if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tlg), bytes) != hipSuccess) return -1;
    } else {
        void *d = nullptr;
        if (hipGetSymbolAddress(&d, HIP_SYMBOL(g_tlg)) != hipSuccess || hipMemset(d, 0, bytes) != hipSuccess) return -1;
    }
    return (long long)bytes;
}
#endif
