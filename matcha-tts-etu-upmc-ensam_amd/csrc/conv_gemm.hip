// Token-major implicit GEMM for every conv / linear of the CFM decoder (gfx950 MFMA).
//
// Reference ops replaced: Conv1d k3/k1 (decoder.py:59,78,95,192,239,248,251), the stride-2 Downsample
// (:95), the ConvTranspose1d(4,2,1) Upsample (:112, run as two phase GEMMs), diffusers Linear layers
// (to_q/k/v, to_out.0, ff.net.0.proj, ff.net.2; transformer.py:155-180) and the time-MLP Linears.
//
// Activations are token-major [rows, C] fp32.  For output row u of batch b, tap j reads input row
// u*in_stride + off[j] of the same batch (zero outside [0, Ti)), times the optional row scale (the
// reference's `x * mask` before every conv).  K = ntaps * cin; every 8-element K chunk lies in one
// tap (cin % 8 == 0).  Weights come packed [N][Kp] (K contiguous, Kp = K rounded up to 8).
// Epilogue: + bias[n] -> erf-GELU -> + residual -> * row scale -> store to row
// b*To_full + u*out_stride + out_off.
//
// Tile: BM = 64*MR rows x BN = 128 cols x BK = 32, 256 threads = 4 waves (2 x 2), each wave owns
// (32*MR) x 64 as MR x 2 tiles of 32x32.  Operands are staged global -> registers -> LDS (the
// gather / mask / fp32->bf16 conversion happens in that pass) with two LDS buffers and one barrier
// per K step: the next tile's global loads are in flight while the current tile's MFMAs run.
//   bf16 path: v_mfma_f32_32x32x16_bf16 (dense bf16 MFMA, fp32 accumulate)
//   fp32 path: v_mfma_f32_32x32x2_f32   (exact fp32 products, the parity mode)
//
// wgrad (conv_wgrad_kernel): dW[n][k] = sum_rows dY[row][n] * A_gathered[row][k], the reduction over
// tokens split across blocks into fp32 partial slabs (deterministic) that reduce.hip sums in a fixed
// order -- at once, or batched with the step's other gradient sums -- together with the bias gradient
// (column sums of dY, accumulated in the k-tile-0 blocks).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include <cstdint>

#include "gemm_epilogue.h"
#include "conv_gemm_wreg.h"
#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p names row q / columns 4p..4p+3 of a 4 x 16 block of
// 16-bit elements and receives column (lane & 15) of the block's 4 rows.  Two reads, rows r..r+3 and
// r+4..r+7, give a lane the 8 reduction-index elements of a 32x32x16 MFMA operand that is stored
// row-major along the reduction index.
__device__ __forceinline__ bf16x8 tr_read8(const uint16_t *p, int row_stride) {
    using LdsS4 = __attribute__((address_space(3))) s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LdsS4 *)(p));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LdsS4 *)(p + 4 * row_stride));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// -DMTTS_PIN_PREFETCH=0 builds the register-staged loops without the scheduling fence (A/B builds)
#ifndef MTTS_PIN_PREFETCH
#define MTTS_PIN_PREFETCH 1
#endif
constexpr bool g_pin_prefetch = MTTS_PIN_PREFETCH != 0;

// -DMTTS_GEMM_TIMELINE=1 (diagnostic builds only, tools/r5/gemm_timeline.py): lane 0 of every wave of the
// register-staged one-step schedule stamps the 100 MHz wall clock at each phase of each K step into g_tl
// ([wave][kTlSlots]: HW ids, start, prologue, then per step: loads issued / MFMAs issued / LDS stored /
// barrier passed, loop end, epilogue end); read back by mtts_gemm_timeline_read.
#ifndef MTTS_GEMM_TIMELINE
#define MTTS_GEMM_TIMELINE 0
#endif
#if MTTS_GEMM_TIMELINE
constexpr int kTlSlots = 128, kTlWaves = 16384, kTlSteps = 30;
__device__ long long g_tl[kTlWaves * kTlSlots];
#define MTTS_TL(slot)                                                                                    \
    do {                                                                                                 \
        const int tl_w = (int)blockIdx.x * (WM * WN) + wave;                                            \
        if (lane == 0 && tl_w < kTlWaves && (slot) < kTlSlots) g_tl[tl_w * kTlSlots + (slot)] = wall_clock64(); \
    } while (0)
#else
#define MTTS_TL(slot) \
    do {              \
    } while (0)
#endif

__device__ __forceinline__ uint16_t to_bf16(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// (a, b) -> one v_cvt_pk_bf16_f32 (two scalar to_bf16 + shift/or were compiled to SDWA repacks)
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}




using mtts::divmod_fast;

constexpr int kBN = 128;
constexpr int kBK = 32;
constexpr int kThreads = 256;

struct Gather {  // per-thread precomputed row info for one staged A row
    int in_base;  // b*Ti (input row base of this batch)
    int in_u;     // u*in_stride
    bool valid;
};

template <bool BF16>
struct Stage;  // LDS element type + padding per precision

template <>
struct Stage<true> {
    using T = uint16_t;
    static constexpr int PAD = 8;  // 80-byte rows: conflict-free ds_read_b128 (16 distinct rows)
};
template <>
struct Stage<false> {
    using T = float;
    static constexpr int PAD = 1;  // 33-dword rows: conflict-free ds_read_b32 column reads
};

// Block = WM x WN waves; each wave owns TM x TN MFMA tiles of 32x32 -> block tile
// BM = 32*WM*TM rows x BN = 32*WN*TN cols, K step KB (32, or 64 for bf16: each step is one global
// round trip, so a longer step halves the exposed latency per MFMA).
// WS (bf16 only, MTTS_GEMM_F_W_SPLIT): W carries a second bf16 plane (the rounding residual of the fp32
// weights) at W + N*Kp; it is staged beside the first and every fragment pair issues two MFMAs.
// AS (with WS, MTTS_GEMM_F_A_SPLIT): the staging pass also writes A's rounding residual bf16(a - bf16(a))
// as a second A plane, and each fragment triple issues A_hi*W_hi, A_hi*W_lo, A_lo*W_hi (bf16x3).
// Split-K (part != NULL, round 4; fp32 schedules): grid = tiles x S with the S splits of a tile adjacent (one
// XCD); split s runs K steps [s * ksteps, min(nk, (s + 1) * ksteps)) and stores its raw fp32 partial tile to
// part[s][M][N]; mtts::splitk_combine (conv_gemm_glds.hip) then sums the splits in order and runs the
// epilogue.  For the text encoder's long reductions on few row tiles (3840 x 192 x 2304: 240 tiles of 72
// K steps at fp32 -- the parity policy's exact-fp32 encoder forward and 32-true).
template <bool BF16, int WM, int WN, int TM, int TN, int KB = kBK, int DEPTH = 1, bool WS = false, bool AS = false>
__global__ __launch_bounds__(64 * WM * WN) void conv_gemm_kernel(mtts_conv_gemm_args p, int ksteps, float *part) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BM = 32 * WM * TM, BN = 32 * WN * TN;
    constexpr int KC = KB / 8;                    // 8-element chunks per staged row
    constexpr int CA = (BM * KC + NT - 1) / NT;  // A chunks per thread per K step
    constexpr int CB = (BN * KC + NT - 1) / NT;  // B chunks per thread per K step
    static_assert(BM * KC % NT == 0 || NT % (BM * KC) == 0, "tile/threads mismatch");
    static_assert(BF16 || KB == kBK, "fp32 path uses 32-wide K steps");
    static_assert(!WS || BF16, "the split weight planes are bf16");
    static_assert(!AS || WS, "the split A planes go with split weights");
    using ST = typename Stage<BF16>::T;
    constexpr int LDK = KB + Stage<BF16>::PAD;
    constexpr int BPL = (BN + 1) * LDK;   // one W plane image
    constexpr int APL = (BM + 1) * LDK;   // one A plane image
    __shared__ ST As[2][(AS ? 2 : 1) * APL];  // + one dummy row: staging target of threads without an A chunk
    __shared__ ST Bs[2][(WS ? 2 : 1) * BPL];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wr = wave / WN, wc = wave % WN;
    const int M = p.nb * p.To;
    // 1-D grid, XCD-contiguous: the dispatcher deals consecutive block ids round-robin over the 8 XCDs,
    // so block id b is relabelled to the (b % 8)-th contiguous run of tiles (bijective for any grid
    // size), and tiles are numbered N-fastest -- every column block of an A row panel runs on the same
    // XCD at about the same time and reads the panel from that XCD's L2
    int m0, n0, kstep0 = 0, nk = (p.K + KB - 1) / KB;
    {
        const int nt = (p.N + BN - 1) / BN;
        const int nwg = gridDim.x, orig = blockIdx.x;
        const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
        int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
        if (part) {  // split-K: the splits of a tile are adjacent
            const int ntiles = ((M + BM - 1) / BM) * nt;
            const int S = nwg / ntiles;
            const int tile = wgid / S, split = wgid - tile * S;
            wgid = tile;
            kstep0 = split * ksteps;
            nk = min(ksteps, nk - kstep0);
        }
        const int mt = wgid / nt;
        m0 = mt * BM;
        n0 = (wgid - mt * nt) * BN;
    }
    const int kbase = kstep0 * KB;  // absolute K offset of this block's first step
    const float inv_to = 1.0f / (float)p.To;

    Gather ga[CA];
    // tap offsets form an arithmetic progression (checked at launch): off_j = off_0 + j*step in scalar
    // registers -- a lookup table (select chain or array) was compiled to a scratch / kernarg load per
    // tap change inside the K loop
    const int off0 = p.off[0], offstep = p.ntaps > 1 ? p.off[1] - p.off[0] : 0;
    auto toff_of = [&](int j) { return off0 + j * offstep; };
    int a_row[CA], a_kc[CA], a_j[CA], a_ch[CA], a_toff[CA];  // (tap, channel, tap offset) at the current step
    bool a_on[CA];                               // this thread stages an A chunk (tiles with BM*4 < NT)
#pragma unroll
    for (int c = 0; c < CA; ++c) {
        const int q = tid + NT * c;
        a_on[c] = q < BM * KC;
        a_row[c] = a_on[c] ? q / KC : BM;  // BM: the dummy row
        a_kc[c] = (q % KC) * 8;
        const int m = m0 + a_row[c];
        ga[c].valid = a_on[c] && m < M;
        int b = 0, u = 0;
        if (ga[c].valid) divmod_fast(m, p.To, inv_to, b, u);
        ga[c].in_base = b * p.Ti;
        ga[c].in_u = u * p.in_stride;
        a_j[c] = (kbase + a_kc[c]) / p.cin;
        a_ch[c] = kbase + a_kc[c] - a_j[c] * p.cin;
        a_toff[c] = toff_of(a_j[c]);
    }
    int b_row[CB], b_kc[CB];
    bool b_on[CB];
#pragma unroll
    for (int c = 0; c < CB; ++c) {
        const int q = tid + NT * c;
        b_on[c] = q < BN * KC;
        b_row[c] = b_on[c] ? q / KC : BN;  // BN: the dummy row
        b_kc[c] = (q % KC) * 8;
    }

    // One staged K step.  Loads are issued unconditionally from clamped (always valid) addresses and
    // the validity / row-mask scale is applied only when the registers are written to LDS: no branch
    // around a load and no use of a loaded value before store_tile, so the loads stay in flight
    // through the compute phase and across the LDS-only barrier (counted vmcnt waits, not vmcnt(0)).
    struct Regs {
        float4 a[CA][2];
        float as[CA];   // raw a_scale value (or junk when a_scale is null)
        bool aok[CA];
        float4 bf[CB][2];
        uint4 bh[CB];
        uint4 bl[WS ? CB : 1];  // WS: the lo plane's chunk
        bool bok[CB];
    };
    Regs R0, R1;  // two steps in flight for DEPTH == 2

    auto load_tile = [&](Regs &R, int k0) {
#pragma unroll
        for (int c = 0; c < CA; ++c) {
            const int k = k0 + a_kc[c];
            const int irow = ga[c].in_u + a_toff[c];
            const bool ok = ga[c].valid && k < p.K && irow >= 0 && irow < p.Ti;
            const size_t r = ok ? (size_t)(ga[c].in_base + irow) : 0;
            const int ch = ok ? a_ch[c] : 0;
            a_ch[c] += KB;  // advance (tap, channel) to the next K step
            if (a_ch[c] >= p.cin) {
                while (a_ch[c] >= p.cin) { a_ch[c] -= p.cin; ++a_j[c]; }
                a_toff[c] = toff_of(a_j[c]);
            }
            const float4 *src = reinterpret_cast<const float4 *>(p.A + r * p.lda + ch);
            R.a[c][0] = src[0];
            R.a[c][1] = src[1];
            R.as[c] = *(p.a_scale ? p.a_scale + r : p.A);
            R.aok[c] = ok;
        }
#pragma unroll
        for (int c = 0; c < CB; ++c) {
            const int n = n0 + b_row[c];
            const int k = k0 + b_kc[c];
            const bool ok = b_on[c] && n < p.N && k < p.Kp;
            const size_t off = ok ? (size_t)n * p.Kp + k : 0;
            if constexpr (BF16) {
                R.bh[c] = *reinterpret_cast<const uint4 *>(static_cast<const uint16_t *>(p.W) + off);
                if constexpr (WS)
                    R.bl[c] = *reinterpret_cast<const uint4 *>(static_cast<const uint16_t *>(p.W) + (size_t)p.N * p.Kp + off);
            } else {
                const float4 *src = reinterpret_cast<const float4 *>(static_cast<const float *>(p.W) + off);
                R.bf[c][0] = src[0];
                R.bf[c][1] = src[1];
            }
            R.bok[c] = ok;
        }
    };

    auto store_tile = [&](const Regs &R, int buf) {
#pragma unroll
        for (int c = 0; c < CA; ++c) {  // unconditional (threads without a chunk write the dummy row)
            const float sc = R.aok[c] ? (p.a_scale ? R.as[c] : 1.0f) : 0.0f;
            const float e[8] = {R.a[c][0].x * sc, R.a[c][0].y * sc, R.a[c][0].z * sc, R.a[c][0].w * sc,
                                R.a[c][1].x * sc, R.a[c][1].y * sc, R.a[c][1].z * sc, R.a[c][1].w * sc};
            ST *dst = &As[buf][a_row[c] * LDK + a_kc[c]];
            if constexpr (BF16) {
                uint4 w;
                w.x = pack_bf16x2(e[0], e[1]);
                w.y = pack_bf16x2(e[2], e[3]);
                w.z = pack_bf16x2(e[4], e[5]);
                w.w = pack_bf16x2(e[6], e[7]);
                *reinterpret_cast<uint4 *>(dst) = w;
                if constexpr (AS) {  // the residual plane: a - bf16(a), exact in fp32, rounded once to bf16
                    const uint32_t hw[4] = {w.x, w.y, w.z, w.w};
                    uint32_t lw[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const float h0 = __uint_as_float(hw[q] << 16), h1 = __uint_as_float(hw[q] & 0xffff0000u);
                        lw[q] = pack_bf16x2(e[2 * q] - h0, e[2 * q + 1] - h1);
                    }
                    *reinterpret_cast<uint4 *>(dst + APL) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) dst[i] = e[i];
            }
        }
#pragma unroll
        for (int c = 0; c < CB; ++c) {
            ST *dst = &Bs[buf][b_row[c] * LDK + b_kc[c]];
            if constexpr (BF16) {
                *reinterpret_cast<uint4 *>(dst) = R.bok[c] ? R.bh[c] : make_uint4(0, 0, 0, 0);
                if constexpr (WS) *reinterpret_cast<uint4 *>(dst + BPL) = R.bok[c] ? R.bl[c] : make_uint4(0, 0, 0, 0);
            } else {
                const float m = R.bok[c] ? 1.f : 0.f;
                const float e[8] = {R.bf[c][0].x * m, R.bf[c][0].y * m, R.bf[c][0].z * m, R.bf[c][0].w * m,
                                    R.bf[c][1].x * m, R.bf[c][1].y * m, R.bf[c][1].z * m, R.bf[c][1].w * m};
#pragma unroll
                for (int i = 0; i < 8; ++i) dst[i] = e[i];
            }
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

    const int lr = lane & 31, lh = lane >> 5;
    auto compute = [&](int buf) {
        if constexpr (BF16) {
#pragma unroll
            for (int ks = 0; ks < KB / 16; ++ks) {
                bf16x8 af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    af[i] = *reinterpret_cast<const bf16x8 *>(
                        &As[buf][(wr * 32 * TM + i * 32 + lr) * LDK + ks * 16 + 8 * lh]);
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    bfr[j] = *reinterpret_cast<const bf16x8 *>(
                        &Bs[buf][(wc * 32 * TN + j * 32 + lr) * LDK + ks * 16 + 8 * lh]);
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
                if constexpr (WS) {
                    bf16x8 bhi[AS ? TN : 1];
                    if constexpr (AS) {
#pragma unroll
                        for (int j = 0; j < TN; ++j) bhi[j] = bfr[j];
                    }
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        bfr[j] = *reinterpret_cast<const bf16x8 *>(
                            &Bs[buf][BPL + (wc * 32 * TN + j * 32 + lr) * LDK + ks * 16 + 8 * lh]);
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
                    if constexpr (AS) {
#pragma unroll
                        for (int i = 0; i < TM; ++i)
                            af[i] = *reinterpret_cast<const bf16x8 *>(
                                &As[buf][APL + (wr * 32 * TM + i * 32 + lr) * LDK + ks * 16 + 8 * lh]);
#pragma unroll
                        for (int i = 0; i < TM; ++i)
#pragma unroll
                            for (int j = 0; j < TN; ++j)
                                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bhi[j], acc[i][j], 0, 0, 0);
                    }
                }
            }
        } else {
#pragma unroll
            for (int ks = 0; ks < kBK / 2; ++ks) {
                float af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) af[i] = As[buf][(wr * 32 * TM + i * 32 + lr) * LDK + ks * 2 + lh];
#pragma unroll
                for (int j = 0; j < TN; ++j) bfr[j] = Bs[buf][(wc * 32 * TN + j * 32 + lr) * LDK + ks * 2 + lh];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        }
    };

    // The scheduling fence after each prefetch keeps its global loads ahead of the step's MFMAs: without it
    // the machine scheduler sank them behind all but the last few MFMAs (ISA of the fp32 64 x 64 schedule,
    // round 5), so the vmcnt wait before store_tile exposed the whole global round trip every step.
    if constexpr (DEPTH == 2) {
        // two K steps in flight: the loads of step kt+2 are issued before computing step kt, stored to
        // LDS after computing step kt+1 -- two compute phases cover each global round trip
        load_tile(R0, kbase);
        store_tile(R0, 0);
        load_tile(R1, kbase + KB);
        mtts::lds_barrier();
        for (int kt = 0; kt < nk; kt += 2) {
            load_tile(R0, kbase + (kt + 2) * KB);
            if (g_pin_prefetch) __builtin_amdgcn_sched_barrier(0);
            compute(0);
            store_tile(R1, 1);
            mtts::lds_barrier();
            if (kt + 1 >= nk) break;
            load_tile(R1, kbase + (kt + 3) * KB);
            if (g_pin_prefetch) __builtin_amdgcn_sched_barrier(0);
            compute(1);
            store_tile(R0, 0);
            mtts::lds_barrier();
        }
    } else {
        // branch-free body (no phi copies of in-flight registers): the step after the last one loads
        // clamped addresses with every chunk masked off and stores into the unused buffer
#if MTTS_GEMM_TIMELINE
        if (lane == 0 && (int)blockIdx.x * (WM * WN) + wave < kTlWaves)
            g_tl[((int)blockIdx.x * (WM * WN) + wave) * kTlSlots] =
                ((long long)__smid() << 32) | (long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        MTTS_TL(1);
#endif
        load_tile(R0, kbase);
        store_tile(R0, 0);
        mtts::lds_barrier();
        MTTS_TL(2);
        for (int kt = 0; kt < nk; ++kt) {
            load_tile(R0, kbase + (kt + 1) * KB);
            if (g_pin_prefetch) __builtin_amdgcn_sched_barrier(0);
#if MTTS_GEMM_TIMELINE
            if (kt < kTlSteps) MTTS_TL(3 + 4 * kt);
#endif
            compute(kt & 1);
#if MTTS_GEMM_TIMELINE
            __builtin_amdgcn_sched_barrier(0);
            if (kt < kTlSteps) MTTS_TL(4 + 4 * kt);
#endif
            store_tile(R0, (kt + 1) & 1);
#if MTTS_GEMM_TIMELINE
            if (kt < kTlSteps) MTTS_TL(5 + 4 * kt);
#endif
            mtts::lds_barrier();
#if MTTS_GEMM_TIMELINE
            if (kt < kTlSteps) MTTS_TL(6 + 4 * kt);
#endif
        }
        MTTS_TL(kTlSlots - 2);
    }

    // ---- epilogue ---- (the K loop ended with a barrier after every wave's last LDS access: Bs is free
    // for the 16-byte-row epilogue's per-wave 4 KiB staging images when it is large enough)
    if constexpr (sizeof(Bs) >= (size_t)WM * WN * 4096) {
        if (part) {  // split-K partial (the launcher only splits when Bs holds the staging images)
            mtts::gemm_store_partial<TM, TN>(p, acc, reinterpret_cast<float *>(reinterpret_cast<unsigned char *>(&Bs[0][0]) + wave * 4096),
                                             part + (size_t)(kstep0 / ksteps) * M * p.N, m0 + wr * 32 * TM, n0 + wc * 32 * TN,
                                             lane);
            MTTS_TL(kTlSlots - 1);
            return;
        }
        if (mtts::gemm_epilogue_vec_ok(p)) {
            mtts::gemm_epilogue_vec<TM, TN>(p, acc, reinterpret_cast<float *>(reinterpret_cast<unsigned char *>(&Bs[0][0]) + wave * 4096),
                                            m0 + wr * 32 * TM, n0 + wc * 32 * TN, lane);
            MTTS_TL(kTlSlots - 1);
            return;
        }
    }
    mtts::gemm_epilogue<TM, TN>(p, acc, m0 + wr * 32 * TM, n0 + wc * 32 * TN, lr, lh);
}

// ------------------------------------------------------------------------------------------------
// wgrad: partial[s][n][k] = sum over the split's rows of dY[row][n] * A_gathered[row][k]
// Tile 128 (n) x 128 (k), 4 waves of 64 x 64; the reduction dim (token rows) advances KB rows per
// step, double-buffered with a one-step register prefetch (one barrier per step).  A thread stages
// row PAIRS x 4 columns.  bf16: both operands are staged row-major ([row][col], one conflict-free
// ds_write_b64 per row and operand) with 80-dword rows and read with ds_read_b64_tr_b16 (row stride
// = 16 mod 64 dwords: the 4 rows a 32-lane half reads sit on disjoint banks).  fp32: staged
// transposed ([col][row], 33-dword rows, conflict-free ds_read_b32 column reads).  k-tile-0 blocks
// also sum dY columns (bias grad) in a fixed order.
template <bool BF16, int KB>
struct WgradGeom {
    static constexpr int T = 128;
    static constexpr int LDR = KB + Stage<BF16>::PAD;  // fp32: row stride of the transposed images
    static constexpr int LDW = T + 32;                  // bf16: row stride of the row-major images
    static constexpr int kImg = BF16 ? KB * LDW : T * LDR;  // elements per operand image
    static constexpr int CH = KB * 16 / kThreads;       // (2 rows x 4 cols) chunks per thread per operand
    using ST = typename Stage<BF16>::T;
    static constexpr size_t kBufBytes = (size_t)2 * kImg * sizeof(ST);  // Ys + Xs of one stage
    static constexpr size_t kLds = 2 * kBufBytes;
    static_assert((size_t)(KB / 2) * T * sizeof(float) <= kLds, "db scratch fits the operand buffers");
};

// INC: rows advance by exactly KB per load call, so each staged row's (u, dY offset, A row) is
// updated incrementally -- an add and one wrap select instead of a division and 64-bit address math
// per row and step (the loop was VALU-bound: ~365 VALU vs 8 MFMA per step).  Requires To >= KB (one
// wrap per step) and 32-bit element offsets; the launcher picks the generic path otherwise.
// ABF16: A holds bf16 (MTTS_GEMM_F_A_BF16, bf16 precision only): 8-byte row chunks instead of 16, no
// conversion on the way to LDS (the masked-row zeroing is a select).
// YBF16: dY holds bf16 (MTTS_WGRAD_F_DY_BF16): 8-byte row chunks, staged as is (the bias column sums
// convert exactly).
// LIN (with INC): stride 1, Ti == To == To_full, no output offset -- the dY row of token row m is m and
// its tap-j A row m + off_j, so the per-step address advance is one uniform offset (rb * ld) and only
// the tap validity needs the row's position u in its sequence (~12 instead of ~22 vector instructions
// per staged row; the bias column sums only in the k-tile-0 blocks, behind a block-uniform branch).
// HV = 2: two 4-wave halves per workgroup reduce the two halves of the split's row range into the same
// 128 x 128 tile (own LDS rings, one shared barrier sequence: both halves run the same step count, rows
// past their range masked), then add (half 0 + half 1, fixed order) before ONE slab write: the same waves
// per CU as twice the workgroups, half the partial slabs that the step's batched reduce re-reads.
// Batched launch: up to kWgradBatch independent weight gradients of the same kernel instantiation in one
// grid (the blocks of job j are [first[j], first[j+1]); each job keeps its own row split, so a job's
// partial slabs are bitwise those of its own launch).  The backward's queued weight gradients run this
// way (mtts::flush_wgrads) instead of one latency-bound launch per layer; a lone call is a batch of one.
struct WgradJobK {
    mtts_conv_wgrad_args a;
    float *part, *part_db;  // the job's slabs [splits][N][K] and bias partials [splits][N] (or null)
    int32_t rps;            // token rows per split
    int32_t splits;
    // in-kernel split sum (cnt != null): per-tile arrival counters (zero at rest) and where the sums go --
    // dW[n*sn + c*sc + j*sj] for reduction column k = j*cin + c, db[n] -- (+=) when accumulate
    int32_t *cnt;
    float *dw, *db;
    int64_t sn, sc, sj;
    int32_t accumulate;
    int32_t pad_;
};

// The last block of a tile to arrive sums the tile's split slabs in split order and writes dW (and db):
// every block's slab stores are published by an agent-scope release before its ticket (fetch_add on the
// tile's counter); the last arriver acquires, reads every slab with plain vector loads, and re-zeroes the
// counter.  The sum order is fixed (split 0, 1, ...) whatever the arrival order: deterministic, and no
// separate reduce launch or its re-read of the slabs from HBM.
__device__ __forceinline__ void wgrad_combine(const WgradJobK &J, int tile, int n0, int k0, bool ktile0) {
    __shared__ int s_last;
    const mtts_conv_wgrad_args &p = J.a;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab / db stores have completed
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = __hip_atomic_fetch_add(J.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == J.splits - 1;
    }
    __syncthreads();
    if (!s_last) return;  // block-uniform
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const size_t NK = (size_t)p.N * p.K;
    const int nthr = (int)blockDim.x;
    // 128 x 128 tile as float4 groups along k (K = ntaps * cin, cin % 8 == 0: a group is all in or out)
    for (int g = (int)threadIdx.x; g < 128 * 32; g += nthr) {
        const int n = n0 + (g >> 5), k = k0 + (g & 31) * 4;
        if (n >= p.N || k >= p.K) continue;
        const float *src = J.part + (size_t)n * p.K + k;
        float4 a = *reinterpret_cast<const float4 *>(src);
        for (int sp = 1; sp < J.splits; ++sp) {
            const float4 b = *reinterpret_cast<const float4 *>(src + sp * NK);
            a.x += b.x;
            a.y += b.y;
            a.z += b.z;
            a.w += b.w;
        }
        const float v[4] = {a.x, a.y, a.z, a.w};
        const int j0 = k / p.cin, c0 = k - j0 * p.cin;  // the group lies inside one tap (cin % 4 == 0)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float *o = J.dw + n * J.sn + (int64_t)(c0 + e) * J.sc + (int64_t)j0 * J.sj;
            *o = J.accumulate ? *o + v[e] : v[e];
        }
    }
    if (ktile0 && J.part_db && J.db) {
        for (int x = (int)threadIdx.x; x < 128; x += nthr) {
            const int n = n0 + x;
            if (n >= p.N) continue;
            float a = J.part_db[n];
            for (int sp = 1; sp < J.splits; ++sp) a += J.part_db[(size_t)sp * p.N + n];
            J.db[n] = J.accumulate ? J.db[n] + a : a;
        }
    }
    if (threadIdx.x == 0) __hip_atomic_store(J.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int kWgradBatch = 12;  // ~1.7 KiB of kernel arguments
struct WgradBatch {
    WgradJobK job[kWgradBatch];
    int32_t first[kWgradBatch + 1];
    int32_t njobs;
};

// One (tile, split) block of a batch: vb is its index in the batch's block numbering.
template <bool BF16, int KB, int DEPTH, bool INC, bool ABF16, bool YBF16, bool LIN, int HV>
__device__ __forceinline__ void wgrad_block(const WgradBatch &wb, const int vb) {
    int jb = 0;  // this block's job (block-uniform scan over the batch's first-block table)
    while (jb + 1 < wb.njobs && vb >= wb.first[jb + 1]) ++jb;
    const mtts_conv_wgrad_args &p = wb.job[jb].a;
    const int rows_per_split = wb.job[jb].rps;
    float *__restrict__ part = wb.job[jb].part;
    float *__restrict__ part_db = wb.job[jb].part_db;
    const int blk = vb - wb.first[jb], nblk = wb.first[jb + 1] - wb.first[jb];
    static_assert(HV == 1 || (HV == 2 && DEPTH == 1), "two halves: one step in flight");
    static_assert(HV == 1 || (size_t)64 * kThreads * sizeof(float) <= 2 * WgradGeom<BF16, KB>::kLds,
                  "half 1's accumulators fit the two halves' LDS");
    static_assert(!ABF16 || BF16, "bf16 A needs the bf16 path");
    static_assert(!YBF16 || BF16, "bf16 dY needs the bf16 path");
    static_assert(!LIN || INC, "the linear row walk is a special case of the incremental one");
    const uint16_t *A16 = reinterpret_cast<const uint16_t *>(p.A);
    const uint16_t *Y16 = reinterpret_cast<const uint16_t *>(p.dY);
    using Gm = WgradGeom<BF16, KB>;
    using ST = typename Gm::ST;
    constexpr int T = Gm::T, LDR = Gm::LDR, LDW = Gm::LDW, IMG = Gm::kImg, CH = Gm::CH;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int hv = HV == 2 ? (int)(threadIdx.x >> 8) : 0;  // this thread's half
    ST *Ybuf = reinterpret_cast<ST *>(smem) + hv * 4 * IMG;  // per half: [2][IMG] then Xs [2][IMG]
    ST *Xbuf = Ybuf + 2 * IMG;

    const int tid = (int)threadIdx.x & (kThreads - 1), lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int lr = lane & 31, lh = lane >> 5;
    // 1-D grid relabelled XCD-contiguous (as conv_gemm_kernel), tiles numbered n-fastest, then k, then
    // split: the tiles of one split read the same token rows and now share one XCD's L2
    int n0, k0, split, ktile;
    {
        const int ntn = (p.N + T - 1) / T, ntk = (p.K + T - 1) / T;
        const int nwg = nblk, orig = blk;  // the job's own block numbering (its launch alone: the grid's)
        const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
        const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
        split = wgid / (ntn * ntk);
        const int t = wgid - split * ntn * ntk;
        ktile = t / ntn;
        n0 = (t - ktile * ntn) * T;
        k0 = ktile * T;
    }
    const int M = p.nb * p.To;
    // HV = 2: rows_per_split is a multiple of 2 KB; half h takes [split start + h * rows / 2, + rows / 2)
    const int h_rows = rows_per_split / HV;
    const int r_begin = split * rows_per_split + hv * h_rows;
    const int r_end = min(M, r_begin + h_rows);
    const bool do_db = (ktile == 0) && part_db != nullptr;
    const float inv_to = 1.0f / (float)p.To;

    // per-chunk constants: row pair, column group, and the A gather's (tap offset, channel) -- k is
    // fixed per chunk, so no division in the loop
    int c_rp[CH], c_cc[CH], c_toff[CH], c_ch[CH];
    bool c_kok[CH], c_nok[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int q = tid + kThreads * c;
        c_rp[c] = q >> 5;
        c_cc[c] = (q & 31) * 4;
        const int k = k0 + c_cc[c], n = n0 + c_cc[c];
        c_kok[c] = k < p.K;
        const int j = c_kok[c] ? k / p.cin : 0;
        c_ch[c] = c_kok[c] ? k - j * p.cin : 0;  // columns past K / N are never stored: any valid address
        c_toff[c] = mtts::tap_off(p, j);
        c_nok[c] = n < p.N;  // N % 4 == 0: a 4-column group is all in or all out
    }
    // INC state of each staged row (chunk c, row h of the pair) for the NEXT load call
    int s_u[CH][2], s_y[CH][2], s_x[CH][2], s_i[CH][2];
    const int y_step = KB * p.out_stride * p.ldy, y_wrap = (p.To_full - p.To * p.out_stride) * p.ldy;
    const int x_step = KB * p.in_stride, x_wrap = p.Ti - p.To * p.in_stride, i_wrap = -p.To * p.in_stride;
    if constexpr (INC) {
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                int b = 0, u = 0;
                divmod_fast(min(r_begin + 2 * c_rp[c] + h, M - 1), p.To, inv_to, b, u);
                s_u[c][h] = u;
                s_y[c][h] = (b * p.To_full + u * p.out_stride + p.out_off) * p.ldy;
                s_i[c][h] = u * p.in_stride + c_toff[c];
                s_x[c][h] = b * p.Ti + s_i[c][h];
            }
    }
    const int y_col = min(n0 + c_cc[0], p.N - 4);  // per-chunk y column (chunks differ only in row pair)
    // LIN: per staged row, the lane-constant parts of its dY / A element offsets and mask index
    int l_y[LIN ? CH : 1][2], l_x[LIN ? CH : 1][2], l_m[LIN ? CH : 1][2];
    if constexpr (LIN) {
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int rr = 2 * c_rp[c] + h;
                l_y[c][h] = rr * p.ldy + y_col;
                l_m[c][h] = rr + c_toff[c];
                l_x[c][h] = l_m[c][h] * p.lda + c_ch[c];
            }
    }

    // One staged step, loaded unconditionally from clamped addresses; validity, the row mask and the
    // bias column sums are applied at store time so the loads stay in flight through the compute.
    struct Regs {
        float4 y[CH][2], x[CH][2];
        uint2 x16[CH][2];  // ABF16: the 4 bf16 of the chunk
        uint2 y16[CH][2];  // YBF16
        float xs[CH][2];
        bool yok[CH][2], xok[CH][2];
    };
    Regs R0, R1;  // DEPTH 2: two row steps in flight
    float colsum[CH][4];
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) colsum[c][i] = 0.f;

    auto load = [&](Regs &R, int rb) {
        if constexpr (LIN) {
            const int rows_left = r_end - rb;
            const int yb = rb * p.ldy, xb = rb * p.lda;  // uniform
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const bool mv = 2 * c_rp[c] + h < rows_left;
                    const uint32_t ye = (uint32_t)(mv ? yb + l_y[c][h] : y_col);
                    if constexpr (YBF16) R.y16[c][h] = *reinterpret_cast<const uint2 *>(Y16 + ye);
                    else R.y[c][h] = *reinterpret_cast<const float4 *>(p.dY + ye);
                    R.yok[c][h] = mv;
                    const bool xok = mv && (unsigned)(s_u[c][h] + c_toff[c]) < (unsigned)p.Ti;
                    const uint32_t xe = (uint32_t)(xok ? xb + l_x[c][h] : c_ch[c]);
                    if constexpr (ABF16) R.x16[c][h] = *reinterpret_cast<const uint2 *>(A16 + xe);
                    else R.x[c][h] = *reinterpret_cast<const float4 *>(p.A + xe);
                    R.xs[c][h] = *(p.a_scale ? p.a_scale + (uint32_t)(xok ? rb + l_m[c][h] : 0) : p.A);
                    R.xok[c][h] = xok;
                    const int u = s_u[c][h] + KB;
                    s_u[c][h] = u >= p.To ? u - p.To : u;
                }
            return;
        }
        if constexpr (INC) {
            const int rows_left = r_end - rb;
#pragma unroll
            for (int c = 0; c < CH; ++c)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const bool mv = 2 * c_rp[c] + h < rows_left;
                    if constexpr (YBF16)
                        R.y16[c][h] = *reinterpret_cast<const uint2 *>(Y16 + (uint32_t)((mv ? s_y[c][h] : 0) + y_col));
                    else
                        R.y[c][h] = *reinterpret_cast<const float4 *>(p.dY + (uint32_t)((mv ? s_y[c][h] : 0) + y_col));
                    R.yok[c][h] = mv;
                    const bool xok = mv && (unsigned)s_i[c][h] < (unsigned)p.Ti;
                    const int xr = xok ? s_x[c][h] : 0;
                    if constexpr (ABF16)
                        R.x16[c][h] = *reinterpret_cast<const uint2 *>(A16 + (uint32_t)(xr * p.lda + c_ch[c]));
                    else
                        R.x[c][h] = *reinterpret_cast<const float4 *>(p.A + (uint32_t)(xr * p.lda + c_ch[c]));
                    R.xs[c][h] = *(p.a_scale ? p.a_scale + (uint32_t)xr : p.A);
                    R.xok[c][h] = xok;
                    int u = s_u[c][h] + KB;
                    const bool wrap = u >= p.To;
                    s_u[c][h] = wrap ? u - p.To : u;
                    s_y[c][h] += y_step + (wrap ? y_wrap : 0);
                    s_x[c][h] += x_step + (wrap ? x_wrap : 0);
                    s_i[c][h] += x_step + (wrap ? i_wrap : 0);
                }
            return;
        }
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int m = rb + 2 * c_rp[c] + h;
                const bool mv = m < r_end;
                int b = 0, u = 0;
                divmod_fast(mv ? m : 0, p.To, inv_to, b, u);
                const bool yok = mv && c_nok[c];
                const size_t yrow = yok ? (size_t)b * p.To_full + (size_t)u * p.out_stride + p.out_off : 0;
                if constexpr (YBF16)
                    R.y16[c][h] = *reinterpret_cast<const uint2 *>(Y16 + yrow * p.ldy + (yok ? n0 + c_cc[c] : 0));
                else
                    R.y[c][h] = *reinterpret_cast<const float4 *>(p.dY + yrow * p.ldy + (yok ? n0 + c_cc[c] : 0));
                R.yok[c][h] = yok;
                const int irow = u * p.in_stride + c_toff[c];
                const bool xok = mv && c_kok[c] && irow >= 0 && irow < p.Ti;
                const size_t r = xok ? (size_t)b * p.Ti + irow : 0;
                if constexpr (ABF16)
                    R.x16[c][h] = *reinterpret_cast<const uint2 *>(A16 + r * p.lda + (xok ? c_ch[c] : 0));
                else
                    R.x[c][h] = *reinterpret_cast<const float4 *>(p.A + r * p.lda + (xok ? c_ch[c] : 0));
                R.xs[c][h] = *(p.a_scale ? p.a_scale + r : p.A);
                R.xok[c][h] = xok;
            }
    };
    auto store = [&](const Regs &R, int buf) {
        ST *Ys = Ybuf + buf * IMG, *Xs = Xbuf + buf * IMG;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            float yv[2][4], xv[2][4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                // the dY row validity is a SELECT, not a multiply by a 0/1 mask: built with packed-fp32
                // VALU ops, hipcc turned that multiply into v_pk_mul_f32 over the mask pair of two rows
                // (op_sel:[0,1] op_sel_hi:[1,0]), which returned wrong, nondeterministic products under
                // CU co-residency (tools/gpu_r2d.sh reproduces it, variant F fixes it)
                const bool yk = R.yok[c][h];
                const float xm = R.xok[c][h] ? (p.a_scale ? R.xs[c][h] : 1.f) : 0.f;
                float4 yf;
                if constexpr (YBF16) {  // bf16 -> fp32 is exact: the bits move to the high half
                    const uint2 q = R.y16[c][h];
                    yf = make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                                     __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u));
                } else {
                    yf = R.y[c][h];
                }
                yv[h][0] = yk ? yf.x : 0.f; yv[h][1] = yk ? yf.y : 0.f;
                yv[h][2] = yk ? yf.z : 0.f; yv[h][3] = yk ? yf.w : 0.f;
                if constexpr (!ABF16) {
                    xv[h][0] = R.x[c][h].x * xm; xv[h][1] = R.x[c][h].y * xm;
                    xv[h][2] = R.x[c][h].z * xm; xv[h][3] = R.x[c][h].w * xm;
                }
            }
            // INC / generic: unconditional (only k-tile-0 blocks store it; a select per element costs more
            // than the add); LIN: behind the block-uniform branch
            if (!LIN || do_db) {
#pragma unroll
                for (int i = 0; i < 4; ++i) colsum[c][i] += yv[0][i] + yv[1][i];
            }
            const int r2 = 2 * c_rp[c];
            if constexpr (BF16) {
                auto pk = [](float a, float b) { return pack_bf16x2(a, b); };
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    *reinterpret_cast<uint2 *>(&Ys[(r2 + h) * LDW + c_cc[c]]) =
                        make_uint2(pk(yv[h][0], yv[h][1]), pk(yv[h][2], yv[h][3]));
                    if constexpr (ABF16) {  // 0/1 row scale on bf16 A: keep or zero the raw bits
                        const float xm = R.xok[c][h] ? (p.a_scale ? R.xs[c][h] : 1.f) : 0.f;
                        *reinterpret_cast<uint2 *>(&Xs[(r2 + h) * LDW + c_cc[c]]) =
                            xm != 0.f ? R.x16[c][h] : make_uint2(0u, 0u);
                    } else {
                        *reinterpret_cast<uint2 *>(&Xs[(r2 + h) * LDW + c_cc[c]]) =
                            make_uint2(pk(xv[h][0], xv[h][1]), pk(xv[h][2], xv[h][3]));
                    }
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int col = c_cc[c] + i;
                    Ys[col * LDR + r2] = yv[0][i];
                    Ys[col * LDR + r2 + 1] = yv[1][i];
                    Xs[col * LDR + r2] = xv[0][i];
                    Xs[col * LDR + r2 + 1] = xv[1][i];
                }
            }
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

    auto compute = [&](int buf) {
        const ST *Ys = Ybuf + buf * IMG, *Xs = Xbuf + buf * IMG;
        if constexpr (BF16) {
            // this lane's tr-read address inside a 16-row x 32-column operand block
            const int g = lane >> 4;
            const int tro = (8 * (g >> 1) + ((lane >> 2) & 3)) * LDW + 16 * (g & 1) + 4 * (lane & 3);
#pragma unroll
            for (int ks = 0; ks < KB / 16; ++ks) {
                bf16x8 af[2], bfr[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) af[i] = tr_read8(&Ys[ks * 16 * LDW + wr * 64 + i * 32 + tro], LDW);
#pragma unroll
                for (int j = 0; j < 2; ++j) bfr[j] = tr_read8(&Xs[ks * 16 * LDW + wc * 64 + j * 32 + tro], LDW);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int ks = 0; ks < KB / 2; ++ks) {
                float af[2], bfr[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) af[i] = Ys[(wr * 64 + i * 32 + lr) * LDR + ks * 2 + lh];
#pragma unroll
                for (int j = 0; j < 2; ++j) bfr[j] = Xs[(wc * 64 + j * 32 + lr) * LDR + ks * 2 + lh];
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        }
    };

    if constexpr (HV == 2) {
        // both halves: the same step count (block-wide barriers), rows past r_end masked by load()
        load(R0, r_begin);
        int buf = 0;
        for (int s = 0; s < h_rows / KB; ++s) {
            const int rb = r_begin + s * KB;
            store(R0, buf);
            mtts::lds_barrier();
            load(R0, rb + KB);
            if (g_pin_prefetch) __builtin_amdgcn_sched_barrier(0);
            compute(buf);
            buf ^= 1;
        }
        // half 1's accumulators -> LDS (lane-fastest: conflict-free), half 0 adds them: acc0 + acc1
        float *xs = reinterpret_cast<float *>(smem);
        __syncthreads();
        if (hv == 1) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int v = 0; v < 16; ++v) xs[((i * 2 + j) * 16 + v) * kThreads + tid] = acc[i][j][v];
        }
        __syncthreads();
        if (hv == 0) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int v = 0; v < 16; ++v) acc[i][j][v] += xs[((i * 2 + j) * 16 + v) * kThreads + tid];
        }
    } else if (r_begin < r_end) {
        if constexpr (DEPTH == 2) {
            load(R0, r_begin);
            load(R1, r_begin + KB);
            store(R0, 0);
            mtts::lds_barrier();
            for (int rb = r_begin; rb < r_end; rb += 2 * KB) {
                load(R0, rb + 2 * KB);
                if (g_pin_prefetch) __builtin_amdgcn_sched_barrier(0);
                compute(0);
                store(R1, 1);
                mtts::lds_barrier();
                if (rb + KB >= r_end) break;
                load(R1, rb + 3 * KB);
                if (g_pin_prefetch) __builtin_amdgcn_sched_barrier(0);
                compute(1);
                store(R0, 0);
                mtts::lds_barrier();
            }
        } else {
            load(R0, r_begin);
            int buf = 0;
            for (int rb = r_begin; rb < r_end; rb += KB) {
                store(R0, buf);  // buf was last read two steps ago, before the previous barrier
                mtts::lds_barrier();
                load(R0, rb + KB);  // unconditional: past r_end every row is masked off (branch-free body)
                if (g_pin_prefetch) __builtin_amdgcn_sched_barrier(0);
                compute(buf);
                buf ^= 1;
            }
        }
    }

    float *slab = part + (size_t)split * p.N * p.K;
#pragma unroll
    for (int i = 0; i < 2 && hv == 0; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int k = k0 + wc * 64 + j * 32 + lr;
            if (k >= p.K) continue;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int n = n0 + wr * 64 + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * lh;
                if (n < p.N) slab[(size_t)n * p.K + k] = acc[i][j][v];
            }
        }
    if (do_db) {
        // (row pair, column) partial sums -> LDS scratch (reusing the operand buffers), then a fixed-order
        // sum over the KB/2 row pairs (deterministic, no float atomics)
        float *dbs = reinterpret_cast<float *>(smem);  // [HV][KB/2][T]
        __syncthreads();
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int i = 0; i < 4; ++i) dbs[(hv * (KB / 2) + c_rp[c]) * T + c_cc[c] + i] = colsum[c][i];
        __syncthreads();
        for (int x = (int)threadIdx.x; x < T; x += kThreads * HV) {
            const int n = n0 + x;
            float sacc = 0.f;
            for (int g = 0; g < HV * (KB / 2); ++g) sacc += dbs[g * T + x];
            if (n < p.N) part_db[(size_t)split * p.N + n] = sacc;
        }
    }
    if (wb.job[jb].cnt) {
        const int ntn = (p.N + T - 1) / T;
        wgrad_combine(wb.job[jb], ktile * ntn + n0 / T, n0, k0, ktile == 0);
    }
}

// The batch's blocks on gridDim.x workgroups: one each when the grid covers them (the default), else a
// workgroup walks several (a capped grid leaves CUs to a concurrent stream: the side-stream flush, see
// mtts_wgrad_flush_cap).  Whole-block-uniform loop; the barrier protects the LDS images between blocks.
template <bool BF16, int KB, int DEPTH, bool INC, bool ABF16 = false, bool YBF16 = false, bool LIN = false, int HV = 1>
__global__ __launch_bounds__(kThreads * HV) void conv_wgrad_kernel(const WgradBatch wb) {
    const int total = wb.first[wb.njobs];
    for (int vb = (int)blockIdx.x; vb < total; vb += (int)gridDim.x) {
        wgrad_block<BF16, KB, DEPTH, INC, ABF16, YBF16, LIN, HV>(wb, vb);
        __syncthreads();
    }
}

// The GEMM kernels compute tap offsets as off[0] + j*(off[1]-off[0]).
bool taps_arithmetic(const int32_t *off, int ntaps) {
    for (int j = 2; j < ntaps; ++j)
        if (off[j] - off[j - 1] != off[1] - off[0]) return false;
    return true;
}

int check_gather(const void *A, int lda, int cin, int ntaps, int K) {
    if (!A) return mtts::fail(MTTS_ERR_INVALID_ARG, "conv_gemm: A is null");
    if (cin <= 0 || cin % 8 || lda % 4 || (uintptr_t)A % 16)
        return mtts::fail(MTTS_ERR_SHAPE, "conv_gemm: cin must be a multiple of 8, lda of 4, A 16-byte aligned");
    if (ntaps < 1 || ntaps > MTTS_CONV_MAX_TAPS) return mtts::fail(MTTS_ERR_SHAPE, "conv_gemm: 1..8 taps");
    if (K != ntaps * cin) return mtts::fail(MTTS_ERR_SHAPE, "conv_gemm: K != ntaps*cin");
    return MTTS_OK;
}

}  // namespace

// Tile configurations: {WM, WN, TM, TN} -> BM x BN = 32*WM*TM x 32*WN*TN, 64*WM*WN threads.
struct TileCfg {
    int wm, wn, tm, tn, kb, depth = 1;  // depth: K steps in flight in registers (2: bf16 only)
};
constexpr TileCfg kCfgs[] = {
    {2, 2, 1, 2, 32},  // 0: 64 x 128, 256 thr (round-1 default)
    {2, 2, 2, 2, 32},  // 1: 128 x 128, 256 thr
    {1, 2, 1, 1, 32},  // 2: 32 x 64, 128 thr
    {2, 2, 1, 1, 32},  // 3: 64 x 64, 256 thr
    {1, 4, 1, 2, 32},  // 4: 32 x 256, 256 thr
    {2, 4, 1, 2, 32},  // 5: 64 x 256, 512 thr
    {1, 2, 1, 2, 32},  // 6: 32 x 128, 128 thr
    {1, 4, 1, 1, 32},  // 7: 32 x 128, 256 thr (one 32x32 tile per wave)
    {1, 4, 1, 1, 64},  // 8: config 7 with 64-wide K steps (bf16)
    {2, 4, 1, 2, 64},  // 9: config 5 with 64-wide K steps (bf16)
    {2, 2, 1, 2, 64},  // 10: config 0 with 64-wide K steps (bf16)
    {1, 4, 1, 1, 32, 2},  // 11: config 7, two K steps in flight (bf16)
    {1, 4, 1, 1, 64, 2},  // 12: config 8, two K steps in flight (bf16)
    {2, 4, 1, 2, 64, 2},  // 13: config 9, two K steps in flight (bf16)
    {2, 2, 1, 2, 64, 2},  // 14: 64 x 128, K64, two steps in flight (bf16)
    {1, 4, 1, 2, 64, 2},  // 15: 32 x 256, K64, two steps in flight (bf16)
    {2, 2, 1, 1, 64, 2},  // 16: 64 x 64, K64, two steps in flight (bf16)
    {1, 2, 1, 1, 64, 2},  // 17: 32 x 64 (128 threads), K64, two steps in flight (bf16)
    {2, 2, 1, 1, 32, 2},  // 18: config 3 (64 x 64, K32) with two steps in flight (fp32; bf16 too)
};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

namespace mtts {
// conv_gemm_glds.hip: sum part[0..S)[M][N] in split order + the epilogue (splitk_epilogue_kernel)
int splitk_combine(const mtts_conv_gemm_args &p, int M, const float *part, int S, hipStream_t st);
}

template <bool BF16, int C, bool WS = false, bool AS = false>
static void launch_cfg(const mtts_conv_gemm_args &p, int M, hipStream_t st, int splits = 1, float *part = nullptr) {
    constexpr TileCfg c = kCfgs[C];
    constexpr int BM = 32 * c.wm * c.tm, BN = 32 * c.wn * c.tn;
    constexpr int KBc = BF16 ? c.kb : kBK;
    // the split-K partial store stages through the kernel's Bs (as the vector epilogue): it must hold the waves'
    // 4 KiB images, else the launch stays unsplit
    constexpr size_t kBsBytes = (size_t)2 * (WS ? 2 : 1) * (BN + 1) * (KBc + Stage<BF16>::PAD) * sizeof(typename Stage<BF16>::T);
    if (kBsBytes < (size_t)c.wm * c.wn * 4096) splits = 1;
    const int nk = (p.K + KBc - 1) / KBc;
    const int ksteps = splits > 1 ? (nk + splits - 1) / splits : nk;
    const int S = splits > 1 ? (nk + ksteps - 1) / ksteps : 1;  // every split non-empty
    dim3 grid((unsigned)(((M + BM - 1) / BM) * ((p.N + BN - 1) / BN) * S));
    hipLaunchKernelGGL((conv_gemm_kernel<BF16, c.wm, c.wn, c.tm, c.tn, KBc, c.depth, WS, AS>),
                       grid, dim3(64 * c.wm * c.wn), 0, st, p, ksteps, S > 1 ? part : nullptr);
    if (S > 1) mtts::splitk_combine(p, M, part, S, st);
}

// Split-weight (MTTS_GEMM_F_W_SPLIT) register schedules: the two the heuristic picks, 7 (32-wide K steps)
// and 12 (64-wide, two in flight); every other id runs the one with its K step width.  With
// MTTS_GEMM_F_A_SPLIT the same two with the A residual plane (bf16x3).
static void launch_ws(int id, const mtts_conv_gemm_args &p, int M, hipStream_t st) {
    const bool as = p.flags & MTTS_GEMM_F_A_SPLIT;
    if (kCfgs[id].kb == 64) {
        if (as) launch_cfg<true, 12, true, true>(p, M, st);
        else launch_cfg<true, 12, true>(p, M, st);
    } else {
        if (as) launch_cfg<true, 7, true, true>(p, M, st);
        else launch_cfg<true, 7, true>(p, M, st);
    }
}

template <bool BF16>
static void launch_by_id(int id, const mtts_conv_gemm_args &p, int M, hipStream_t st, int splits = 1, float *part = nullptr) {
    if (BF16) splits = 1;  // split-K on the register schedules: fp32 only
    switch (id) {
        case 0: launch_cfg<BF16, 0>(p, M, st, splits, part); break;
        case 1: launch_cfg<BF16, 1>(p, M, st, splits, part); break;
        case 2: launch_cfg<BF16, 2>(p, M, st, splits, part); break;
        case 3: launch_cfg<BF16, 3>(p, M, st, splits, part); break;
        case 4: launch_cfg<BF16, 4>(p, M, st, splits, part); break;
        case 5: launch_cfg<BF16, 5>(p, M, st, splits, part); break;
        case 6: launch_cfg<BF16, 6>(p, M, st, splits, part); break;
        case 7: launch_cfg<BF16, 7>(p, M, st, splits, part); break;
        case 8: launch_cfg<BF16, 8>(p, M, st, splits, part); break;
        case 9: launch_cfg<BF16, 9>(p, M, st, splits, part); break;
        case 10: launch_cfg<BF16, 10>(p, M, st, splits, part); break;
        case 11: launch_cfg<BF16, 11>(p, M, st, splits, part); break;
        case 12: launch_cfg<BF16, 12>(p, M, st, splits, part); break;
        case 13: launch_cfg<BF16, 13>(p, M, st, splits, part); break;
        case 14: launch_cfg<BF16, 14>(p, M, st, splits, part); break;
        case 15: launch_cfg<BF16, 15>(p, M, st, splits, part); break;
        case 16: launch_cfg<BF16, 16>(p, M, st, splits, part); break;
        case 17: launch_cfg<BF16, 17>(p, M, st, splits, part); break;
        default: launch_cfg<BF16, 18>(p, M, st, splits, part); break;
    }
}

// Schedule choice from graph-timed sweeps of the train step's GEMMs WITH their epilogues
// (tools/gemm_sweep2.py -> profiles/r01/gemm_sweep2.log):
//  * erf-GELU / GELU' epilogues (the FFN's 1024-wide projection and its dgrad) are epilogue-bound:
//    the small register-staged 32 x 128 tiles (config 7) keep 3 workgroups per CU so one
//    workgroup's epilogue overlaps another's main loop (75 vs 88 us at 19200 x 1024 x 256);
//  * the LDS-DMA 128 x 256 kernel (8 waves of 64 x 64, 2 stages) when ITS tiles fill the chip in one
//    round and K >= 512 (the 19200-row N = 256 convs / FFN down-projection: 26.9 vs 29.8 us -- W is
//    re-streamed by half as many row tiles);
//  * the LDS-DMA 64 x 256 kernel (3 stages) wins when its tiles fill the chip in ONE round
//    (128..256 tiles, K >= 768: the half-resolution decoder GEMMs, 17.4 vs 19.0 us) -- at 300 tiles
//    the second round's tail makes it lose to config 12;
//  * long reductions on grids far below the CU count (the text encoder's 3840 x 192 x 2304 conv)
//    split K four ways on that kernel (22 vs 29 us);
//  * everything else: 32 x 128 register tiles, 64-wide K steps two in flight (config 12) from
//    K >= 384, 32-wide (config 7) below.  fp32 (parity mode) uses config 7.
static int glds_tiles(const mtts_conv_gemm_args &p, int M) { return ((M + 63) / 64) * ((p.N + 255) / 256); }

static int pick_cfg(const mtts_conv_gemm_args &p, int M, bool bf16) {
    // fp32: 64 x 64 tiles (config 3) on the text encoder's 3840-row GEMMs -- the best register schedule on every
    // one of its exact-fp32 forward calls (tools/r4/gemm_f32_sweep.py, profiles/r04/sweeps/f32_sweep.jsonl: 1044 ->
    // 841 us per step with the split-K counts below); the decoder-sized fp32 GEMMs keep config 7
    // the decoder-sized fp32 GEMMs (32-true) take config 7 with two K steps in flight (config 11): same MFMAs in
    // the same order, 32-true step 16.70 -> 16.50 ms; on the 3840-row encoder GEMMs the two-step 64 x 64 config 18
    // measured no faster (bf16-parity 8.17 vs 8.20 ms; profiles/r04/f32_depth2/).  MTTS_GEMM_F32_DEPTH2=1 / 0:
    // two steps in flight everywhere / nowhere
    static const int d2 = [] { const char *e = getenv("MTTS_GEMM_F32_DEPTH2"); return e ? (e[0] == '1' ? 1 : 0) : -1; }();
    if (!bf16) return M <= 8192 ? (d2 == 1 ? 18 : 3) : (d2 == 0 ? 7 : 11);
    if (p.act == MTTS_ACT_GELU || p.act == MTTS_ACT_DGELU) return 7;
    static const int sched_mask = [] {  // MTTS_GEMM_SCHED_OFF bit mask: A/B switch for experiments
        const char *e = getenv("MTTS_GEMM_SCHED_OFF");
        return e ? atoi(e) : 0;
    }();
    // 128 x 256 LDS-DMA tiles won the isolated sweep on the 19200-row N = 256 GEMMs (26.9 vs 29.8 us) but
    // LOST 0.33 ms per step in an in-step A/B on one box (tools/gpu_ab.sh: 2829 vs 2915 utt/s): opt-in
    if ((sched_mask & 4) && mtts::conv_gemm_glds_applies(p) && p.K >= 512) {  // 128 x 256 tiles, one round
        const int t = ((M + 127) / 128) * ((p.N + 255) / 256);
        if (t >= 128 && t <= 256) return MTTS_GEMM_GLDS + 14;
    }
    if (!(sched_mask & 2) && mtts::conv_gemm_glds_applies(p) && p.K >= 768) {
        const int t = glds_tiles(p, M);
        if ((t >= 128 && t <= 256) || (t < 128 && p.K >= 1536 && p.N % 4 == 0)) return MTTS_GEMM_GLDS + 10;
        // scalar-addressed LDS-DMA loop (whole-tap K steps): 64 x 64 two-stage tiles beat the register
        // schedules on the 19200-row convs (tools/gemm_tall_sweep.py, profiles/r02/gemm_lean: 29.0 vs 29.7,
        // 44.9 vs 48.5, 34.6 vs 38.3 us)
        if (!(sched_mask & 8) && t > 256 && mtts::conv_gemm_glds_lean(p)) return MTTS_GEMM_GLDS + 13;
    }
    if (!(sched_mask & 8) && p.K < 768 && p.N >= 512 && glds_tiles(p, M) >= 256 && mtts::conv_gemm_glds_applies(p) &&
        mtts::conv_gemm_glds_lean(p))
        return MTTS_GEMM_GLDS + 9;  // the decoder's q|k|v projection: 35.1 vs 37.2 us (one workgroup per CU:
                                    // not below one round of tiles -- the text encoder's 3840-row GEMMs)
    return p.K >= 384 ? 12 : 7;
}

// bf16 A (LDS-DMA only): 64 x 256 two-stage tiles when they fill the chip, 64 x 64 three-stage below
// (profiles/r02/gemm_lean: 19.0 vs 21.0 us on the 19200 x 256 x 768 conv, 23.4 vs 32.7 on the q|k|v
// projection; 13.2 vs 13.4 on the 9600-row conv, 16.5 vs 25.5 on the encoder's 3840 x 192 x 2304)
static int pick_cfg_a16(const mtts_conv_gemm_args &p, int M) {
    if (p.act == MTTS_ACT_GELU || p.act == MTTS_ACT_DGELU) return MTTS_GEMM_GLDS + 12;
    return glds_tiles(p, M) >= 256 ? MTTS_GEMM_GLDS + 9 : MTTS_GEMM_GLDS + 12;
}

// Split weight planes (MTTS_GEMM_F_W_SPLIT, the parity policy's decoder forward): W's bytes double, which moves
// the best schedules (step sweep with the split planes, tools/r3/gemm_step_sweep.py SWEEP_PREC=bf16-parity ->
// profiles/r04/sweeps/ws_sweep.jsonl: 2655 -> ~2410 us per step): GELU epilogues keep the 32 x 128 register
// tiles; whole-tap K steps take the LDS-DMA kernels -- 64 x 64 three-stage (bf16 A) / two-stage (fp32 A) on
// the 19200-row N <= 256 GEMMs (31.6 vs 36.0 us, 36.5 vs 56.3), 64 x 256 elsewhere (9600 x 256 x 512: 17.0 vs
// 30.6 on the register schedule the one-plane rule picks below K = 768); other K layouts the 32-wide register
// tiles (19200 x 256 x 480: 32.8 vs 50.6 with 64-wide steps).
static int pick_cfg_ws(const mtts_conv_gemm_args &p, int M) {
    if (p.act == MTTS_ACT_GELU || p.act == MTTS_ACT_DGELU) return 7;
    if (!mtts::conv_gemm_glds_applies(p) || !mtts::conv_gemm_glds_lean(p)) return 7;
    const bool big = M >= 16384 && p.N <= 256;
    if (p.flags & MTTS_GEMM_F_A_BF16) return big ? MTTS_GEMM_GLDS + 12 : MTTS_GEMM_GLDS + 9;
    return M >= 16384 ? MTTS_GEMM_GLDS + 13 : MTTS_GEMM_GLDS + 9;
}

// Split-K (LDS-DMA schedules, heuristic pick only): grids below half the chip with >= 24 K steps
// fp32 register schedule 7 (32 x 128): split K when its tiles fill under one round with >= 48 K steps of 32
// (the text encoder's FFN down-projection, 3840 x 192 x 2304: 240 tiles x 72 steps, 86-98 us unsplit in the
// parity policy's fp32 encoder forward, profiles/r04/fused_wgrad_sum/launches); MTTS_GEMM_F32_SPLITK=0: off
static int pick_splits_f32(const mtts_conv_gemm_args &p, int M, int cfg, int splits) {
    static const bool off = [] { const char *e = getenv("MTTS_GEMM_F32_SPLITK"); return e && e[0] == '0'; }();
    if (p.N % 4 || off || !mtts::gemm_epilogue_vec_ok(p)) return 1;  // the combine is float4
    if (splits > 0) return splits;  // explicit (sweeps): any register schedule
    const int nk = (p.K + kBK - 1) / kBK;
    if (cfg == 3 || cfg == 18) {  // 64 x 64: 4 splits from 28 K steps, 2 from 20 (sweep: 3840 x 192 x 2304 44 us at 4 vs 58 at
                     // 1; k = 5 prenet 27.4 at 4; 3840 x 256 x 768 25.8 at 2; 576-deep ones unsplit)
        const int tiles = ((M + 63) / 64) * ((p.N + 63) / 64);
        if (tiles >= 256 || nk < 20) return 1;
        return nk >= 28 ? 4 : 2;
    }
    if (cfg != 7 && cfg != 11) return 1;
    const int tiles = ((M + 31) / 32) * ((p.N + 127) / 128);
    if (tiles >= 256 || nk < 16) return 1;
    return std::min(8, std::max(2, nk / 9));  // ~9 K steps of 32 per split
}

static int pick_splits(const mtts_conv_gemm_args &p, int M, int cfg, int splits, bool bf16) {
    if (!bf16) return pick_splits_f32(p, M, cfg, splits);
    if (p.flags & MTTS_GEMM_F_SPLIT3) {  // bf16x6 on 64 x 64 LDS-DMA tiles: split K below one round of tiles
        if (cfg < MTTS_GEMM_GLDS || p.N % 4) return 1;
        if (splits > 0) return splits;
        const int tiles = ((M + 63) / 64) * ((p.N + 63) / 64), nk = (p.K + 63) / 64;
        if (tiles >= 256 || nk < 10) return 1;
        return nk >= 24 ? 4 : 2;
    }
    if (cfg < MTTS_GEMM_GLDS || p.N % 4) return 1;
    if (splits > 0) return splits;
    const int nk = (p.K + 63) / 64;
    if (cfg != MTTS_GEMM_GLDS + 10 || glds_tiles(p, M) >= 128 || nk < 24) return 1;
    return 4;
}

struct GemmPlan {
    int cfg, splits;
    size_t ws;
};

static GemmPlan plan_gemm(const mtts_conv_gemm_args &p, bool bf16, int cfg, int splits) {
    const int M = p.nb * p.To;
    if (cfg < 0) cfg = pick_cfg(p, M, bf16);
    if (cfg == MTTS_GEMM_WREG) return {cfg, 1, 0};
    splits = pick_splits(p, M, cfg, splits, bf16);
    size_t ws = 0;
    if (cfg >= MTTS_GEMM_GLDS) {
        ws = mtts::conv_gemm_glds_splitk_bytes(p, splits);
    } else if (splits > 1) {
        const int nk = (p.K + kBK - 1) / kBK, ksteps = (nk + splits - 1) / splits, S = (nk + ksteps - 1) / ksteps;
        ws = S > 1 ? (size_t)S * M * p.N * sizeof(float) : 0;
    }
    return {cfg, splits, ws};
}

// The schedule a call runs: the operand-driven rewrites of an explicit or heuristic config (three weight planes,
// split weight planes, bf16 A, split A).  Shared by the launch and mtts_conv_gemm_workspace_size, so the size
// query plans the schedule -- and the split count -- that will run.  *rc: MTTS_OK or the error.
static int resolve_cfg(const mtts_conv_gemm_args &p, bool bf16, int cfg, int M, int *rc) {
    *rc = MTTS_OK;
    auto err = [&](int code, const char *msg) {
        *rc = mtts::fail(code, msg);
        return cfg;
    };
    if (p.flags & MTTS_GEMM_F_SPLIT3) {  // bf16x6: LDS-DMA 64 x 64 (fp32 A split in the kernel)
        if (!bf16 || (p.flags & (MTTS_GEMM_F_A_BF16 | MTTS_GEMM_F_W_SPLIT | MTTS_GEMM_F_A_SPLIT)))
            return err(MTTS_ERR_INVALID_ARG, "conv_gemm: three weight planes need bf16 precision and an fp32 A");
        if (!mtts::conv_gemm_glds_applies(p))
            return err(MTTS_ERR_UNSUPPORTED, "conv_gemm: three weight planes need the LDS-DMA schedules (cin >= 64)");
        if (cfg < 0) cfg = MTTS_GEMM_GLDS + 12;
        if (cfg < MTTS_GEMM_GLDS) return err(MTTS_ERR_UNSUPPORTED, "conv_gemm: three weight planes need an LDS-DMA schedule");
    }
    // the weight-stationary kernel where its row streams get >= 2 tiles each (or the grid is one round):
    // the K <= 256 linears -- FF up-projection and its GELU' dgrad, q|k|v, the 19200-row projections
    // (tools/r5/gemm_replay.py, profiles/r05/wreg/)
    static const bool wreg_pick = [] { const char *e = getenv("MTTS_GEMM_WREG_PICK"); return !(e && e[0] == '0'); }();
    if (cfg < 0 && bf16 && wreg_pick && mtts::conv_gemm_wreg_applies(p) && mtts::conv_gemm_wreg_preferred(p, M))
        return MTTS_GEMM_WREG;
    static const bool ws_pick = [] { const char *e = getenv("MTTS_GEMM_WS_PICK"); return !(e && e[0] == '0'); }();
    // (a bf16 A goes to the LDS-DMA pick below: pick_cfg_ws may answer a register-staged schedule)
    if (cfg < 0 && bf16 && ws_pick && (p.flags & MTTS_GEMM_F_W_SPLIT) &&
        !(p.flags & (MTTS_GEMM_F_A_SPLIT | MTTS_GEMM_F_A_BF16)))
        cfg = pick_cfg_ws(p, M);
    if (p.flags & MTTS_GEMM_F_A_BF16) {  // bf16 A operands exist only in the LDS-DMA kernels
        if (!bf16 || !mtts::conv_gemm_glds_applies(p))
            return err(MTTS_ERR_UNSUPPORTED,
                              "conv_gemm: a bf16 A needs bf16 precision, cin >= 64, cin / lda % 8 == 0, 0/1 a_scale");
        if (cfg < 0) {
            cfg = pick_cfg_a16(p, M);
        } else if (cfg < MTTS_GEMM_GLDS) {
            return err(MTTS_ERR_UNSUPPORTED, "conv_gemm: a bf16 A needs an LDS-DMA schedule");
        }
    }
    if (p.flags & MTTS_GEMM_F_A_SPLIT) {  // bf16x3: register-staged schedules only (the staging pass splits A)
        if (cfg >= MTTS_GEMM_GLDS) return err(MTTS_ERR_UNSUPPORTED, "conv_gemm: a split A needs a register schedule");
        if (cfg < 0) cfg = p.K >= 384 ? 12 : 7;
    }
    return cfg;
}

static int launch_plan(const mtts_conv_gemm_args &p, bool bf16, const GemmPlan &pl, int M, void *ws, size_t ws_bytes,
                       hipStream_t st) {
    if (pl.cfg == MTTS_GEMM_WREG) return mtts::conv_gemm_wreg_launch(p, M, st);
    if (pl.cfg >= MTTS_GEMM_GLDS) {
        int s = pl.splits;
        if (pl.ws > 0 && (!ws || ws_bytes < pl.ws || (uintptr_t)ws % 16)) s = 1;  // no workspace: unsplit
        return mtts::conv_gemm_glds_launch(pl.cfg - MTTS_GEMM_GLDS, p, M, s, static_cast<float *>(ws), st);
    }
    if (bf16 && (p.flags & MTTS_GEMM_F_W_SPLIT)) launch_ws(pl.cfg, p, M, st);
    else if (bf16) launch_by_id<true>(pl.cfg, p, M, st);
    else {
        int s = pl.splits;
        if (pl.ws == 0 || !ws || ws_bytes < pl.ws || (uintptr_t)ws % 16) s = 1;  // no workspace: unsplit
        launch_by_id<false>(pl.cfg, p, M, st, s, static_cast<float *>(ws));
    }
    return mtts::check_launch("conv_gemm_kernel");
}

static int conv_gemm_impl(const mtts_conv_gemm_args *args, int32_t precision, int cfg, int splits, void *ws,
                          size_t ws_bytes, void *hip_stream) {
    MTTS_CHECK_ARG(args != nullptr, "conv_gemm: args is null");
    const mtts_conv_gemm_args &p = *args;
    int rc = check_gather(p.A, p.lda, p.cin, p.ntaps, p.K);
    if (rc) return rc;
    if (!taps_arithmetic(p.off, p.ntaps))
        return mtts::fail(MTTS_ERR_UNSUPPORTED, "conv_gemm: tap offsets must be an arithmetic progression");
    MTTS_CHECK_ARG(p.W && p.C && p.N > 0 && p.nb >= 0 && p.To >= 0, "conv_gemm: bad output/weights");
    MTTS_CHECK_ARG(p.Kp >= p.K && p.Kp % 8 == 0, "conv_gemm: Kp must be >= K and a multiple of 8");
    MTTS_CHECK_ARG((uintptr_t)p.W % 16 == 0, "conv_gemm: W must be 16-byte aligned");
    MTTS_CHECK_ARG(precision == MTTS_PREC_BF16 || precision == MTTS_PREC_FP32, "conv_gemm: bad precision");
    MTTS_CHECK_ARG(p.act >= MTTS_ACT_NONE && p.act <= MTTS_ACT_DRELU, "conv_gemm: bad act");
    MTTS_CHECK_ARG((p.act != MTTS_ACT_DGELU && p.act != MTTS_ACT_DRELU) || p.aux,
                   "conv_gemm: MTTS_ACT_DGELU / MTTS_ACT_DRELU need aux");
    MTTS_CHECK_ARG(p.dropout_p <= 0.f || (p.seed && p.dropout_p < 1.f), "conv_gemm: dropout needs a seed pointer");
    MTTS_CHECK_ARG(!(p.flags & MTTS_GEMM_F_PRE_BF16) || precision == MTTS_PREC_BF16,
                   "conv_gemm: a bf16 pre-activation needs bf16 precision");
    MTTS_CHECK_ARG(!(p.flags & MTTS_GEMM_F_W_SPLIT) || precision == MTTS_PREC_BF16,
                   "conv_gemm: split weight planes need bf16 precision");
    MTTS_CHECK_ARG(!(p.flags & MTTS_GEMM_F_A_SPLIT) ||
                       ((p.flags & MTTS_GEMM_F_W_SPLIT) && !(p.flags & MTTS_GEMM_F_A_BF16)),
                   "conv_gemm: a split A needs split weight planes and an fp32 A");
    const bool glds_id = cfg >= MTTS_GEMM_GLDS && cfg < MTTS_GEMM_GLDS + mtts::conv_gemm_glds_num_cfgs();
    const bool wreg_id = cfg == MTTS_GEMM_WREG;
    MTTS_CHECK_ARG((cfg >= -1 && cfg < kNumCfgs) || glds_id || wreg_id,
                   "conv_gemm: bad tile config");
    MTTS_CHECK_ARG(splits >= 0, "conv_gemm: bad split count");
    const int M = p.nb * p.To;
    if (M == 0) return MTTS_OK;
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    const bool bf16 = precision == MTTS_PREC_BF16;
    if (wreg_id) {  // weight-stationary schedule, explicit id
        if (!bf16 || !mtts::conv_gemm_wreg_applies(p))
            return mtts::fail(MTTS_ERR_UNSUPPORTED,
                              "conv_gemm: weight-stationary schedule needs bf16, one stride-1 tap, K in {80,160,192,256}");
        return mtts::conv_gemm_wreg_launch(p, M, st);
    }
    if (glds_id && (!bf16 || !mtts::conv_gemm_glds_applies(p)))
        return mtts::fail(MTTS_ERR_UNSUPPORTED, "conv_gemm: LDS-DMA schedule needs bf16, cin >= 64 and a 0/1 a_scale");
    cfg = resolve_cfg(p, bf16, cfg, M, &rc);
    if (rc) return rc;
    const GemmPlan pl = plan_gemm(p, bf16, cfg, splits);
    return launch_plan(p, bf16, pl, M, ws, ws_bytes, st);
}

#if MTTS_GEMM_TIMELINE
// diagnostic builds: copy (or zero, host == NULL) the timeline buffer; returns its size in bytes
extern "C" long long mtts_gemm_timeline_read(void *host) {
    const size_t bytes = sizeof(long long) * kTlWaves * kTlSlots;
    if (host) {
        if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tl), bytes) != hipSuccess) return -1;
    } else {
        void *d = nullptr;
        if (hipGetSymbolAddress(&d, HIP_SYMBOL(g_tl)) != hipSuccess || hipMemset(d, 0, bytes) != hipSuccess) return -1;
    }
    return (long long)bytes;
}
#endif

extern "C" int mtts_conv_gemm(const mtts_conv_gemm_args *args, int32_t precision, void *hip_stream) {
    return conv_gemm_impl(args, precision, -1, 1, nullptr, 0, hip_stream);
}

extern "C" int mtts_conv_gemm_tile(const mtts_conv_gemm_args *args, int32_t precision, int32_t tile_cfg,
                                   void *hip_stream) {
    return conv_gemm_impl(args, precision, tile_cfg, 1, nullptr, 0, hip_stream);
}

extern "C" size_t mtts_conv_gemm_workspace_size(const mtts_conv_gemm_args *args, int32_t precision, int32_t tile_cfg,
                                                int32_t splits) {
    if (!args || args->nb * args->To == 0) return 0;
    const bool bf16 = precision == MTTS_PREC_BF16;
    int rc = MTTS_OK;
    const int cfg = resolve_cfg(*args, bf16, tile_cfg, args->nb * args->To, &rc);
    return rc ? 0 : plan_gemm(*args, bf16, cfg, splits).ws;
}

extern "C" int mtts_conv_gemm_ws(const mtts_conv_gemm_args *args, int32_t precision, int32_t tile_cfg, int32_t splits,
                                 void *workspace, size_t workspace_bytes, void *hip_stream) {
    return conv_gemm_impl(args, precision, tile_cfg, splits, workspace, workspace_bytes, hip_stream);
}

__global__ void dropout_apply_kernel(const float *__restrict__ x, float *__restrict__ y, int rows, int cols, int ld,
                                     float p, const uint32_t *__restrict__ seed) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)rows * cols) return;
    const uint32_t s0 = seed[0], s1 = seed[1];
    const int r = (int)(idx / cols), c = (int)(idx - (int64_t)r * cols);
    const float v = x[(size_t)r * ld + c];
    y[(size_t)r * ld + c] = mtts::dropout_keep(s0, s1, (uint32_t)r, (uint32_t)c, p) ? v * mtts::dropout_scale(p) : 0.f;
}

extern "C" int mtts_dropout_apply(const float *x, float *y, int32_t rows, int32_t cols, int32_t ld, float p,
                                  const uint32_t *seed, void *hip_stream) {
    MTTS_CHECK_ARG(x && y && seed && rows >= 0 && cols >= 0 && ld >= cols && p >= 0.f && p < 1.f,
                   "dropout_apply: bad args");
    const int64_t n = (int64_t)rows * cols;
    if (n == 0) return MTTS_OK;
    hipLaunchKernelGGL(dropout_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(hip_stream), x, y, rows, cols, ld, p, seed);
    return mtts::check_launch("dropout_apply_kernel");
}

// dx = dy * [y > 0] (act RELU) * keep(seed, r, c) / (1-p) (p > 0): the backward of a GEMM epilogue
// "ReLU -> dropout" from its output y (kept and positive <=> pre-activation positive).
__global__ void act_dropout_bwd_kernel(const float *__restrict__ dy, const float *__restrict__ y, float *__restrict__ dx,
                                       int rows, int cols, int ld, int act, float p, const uint32_t *__restrict__ seed,
                                       const float *__restrict__ row_scale) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)rows * cols) return;
    const int r = (int)(idx / cols), c = (int)(idx - (int64_t)r * cols);
    const size_t o = (size_t)r * ld + c;
    float v = dy[o];
    if (row_scale) v = v * row_scale[r];
    if (act == MTTS_ACT_RELU && !(y[o] > 0.f)) v = 0.f;
    if (p > 0.f) v = mtts::dropout_keep(seed[0], seed[1], (uint32_t)r, (uint32_t)c, p) ? v * mtts::dropout_scale(p) : 0.f;
    dx[o] = v;
}

extern "C" int mtts_act_dropout_bwd(const float *dy, const float *y, float *dx, int32_t rows, int32_t cols, int32_t ld,
                                    int32_t act, float p, const uint32_t *seed, void *hip_stream) {
    return mtts_act_dropout_bwd_scaled(dy, y, nullptr, dx, rows, cols, ld, act, p, seed, hip_stream);
}

extern "C" int mtts_act_dropout_bwd_scaled(const float *dy, const float *y, const float *row_scale, float *dx,
                                           int32_t rows, int32_t cols, int32_t ld, int32_t act, float p,
                                           const uint32_t *seed, void *hip_stream) {
    MTTS_CHECK_ARG(dy && dx && rows >= 0 && cols >= 0 && ld >= cols && p >= 0.f && p < 1.f && (p == 0.f || seed),
                   "act_dropout_bwd: bad args");
    MTTS_CHECK_ARG(act == MTTS_ACT_NONE || (act == MTTS_ACT_RELU && y), "act_dropout_bwd: act NONE, or RELU with y");
    const int64_t n = (int64_t)rows * cols;
    if (n == 0) return MTTS_OK;
    hipLaunchKernelGGL(act_dropout_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(hip_stream), dy, y, dx, rows, cols, ld, act, p, seed, row_scale);
    return mtts::check_launch("act_dropout_bwd_kernel");
}

// Split of the token rows over blocks: about target_blocks blocks in total, whole KB-row steps.
constexpr int kWgradMaxTarget = 1024;
// target_blocks < 0: the sweep's rule (tools/wgrad_sweep.py) -- about 768 rows per split (long enough
// to amortize the pipeline and the split's slab write) but never fewer than min_blocks (below).
// batched: the job is queued for a batched launch (mtts::flush_wgrads) whose other jobs fill the chip
// beside it, so it takes fewer, longer splits -- fewer N x K slabs to write and sum (step sweep with the
// whole backward's weight gradients batched at its end, same box: min blocks 384/512 + 768 rows 7.62 ms,
// 256/256 7.41, 128/128 + 768 rows 7.36, 128/128 + 1536 rows 7.34, 64/64 + 3072 rows 7.58).
static void wgrad_plan(const mtts_conv_wgrad_args &p, int kb, int target_blocks, int *splits, int *rows_per_split,
                       int hv = 1, bool batched = false) {
    const int M = p.nb * p.To;
    const int tiles = ((p.N + 127) / 128) * ((p.K + 127) / 128);
    // More blocks keep more row steps in flight per CU (the kernel is latency-bound) but every split adds
    // an N x K fp32 slab that the step's batched reduce reads back.  In-kernel, bf16-stored operands liked
    // ~3 blocks per CU (19200-row conv 49.8 -> 38.4 us, tools/wgrad_store_ab.py), but the whole step --
    // wgrad + its slab reduce -- is fastest at ~2 blocks per CU for bf16 operands and ~1.5 for fp32 ones
    // (same-box step sweep, tools/gpu_ab3.sh: 768/256 8.585 ms, 512/256 8.505, 512/384 8.47, 512/512 8.63,
    // 256/256 8.65; profiles/r02/step_ab_round2b.txt)
    static const int min_blocks = [] { const char *e = getenv("MTTS_WGRAD_MINBLK"); return e ? atoi(e) : 384; }();
    static const int min_blocks16 = [] { const char *e = getenv("MTTS_WGRAD_MINBLK16"); return e ? atoi(e) : 512; }();
    static const int split_rows = [] { const char *e = getenv("MTTS_WGRAD_ROWS"); return e && atoi(e) > 0 ? atoi(e) : 768; }();
    // round 5, with the prefetch fence: 64 minimum blocks per batched job (same box, three alternating rounds:
    // 7.410 / 7.409 / 7.383 vs 7.457 / 7.452 / 7.455 ms at 128; profiles/r05/ab/wgrad_min_blocks_ab.txt) -- the
    // side-stream batch crowds the encoder's backward less
    static const int b_min_blocks = [] { const char *e = getenv("MTTS_WGRAD_BMINBLK"); return e ? atoi(e) : 64; }();
    // round 5: 3072 rows per split in the batched launches (same-box step A/B, tools/r5/gpu_ab_wgrad.sh: 7.604 / 7.583
    // vs 7.611 / 7.631 ms at 1536; 1024 and 4608 slower; profiles/r05/wgrad_split_ab.txt) -- fewer slabs to sum
    static const int b_split_rows = [] { const char *e = getenv("MTTS_WGRAD_BROWS"); return e && atoi(e) > 0 ? atoi(e) : 3072; }();
    // hv = 2: two-half workgroups (twice the waves each): half the workgroups, rows in whole double steps
    const int mb = (batched ? b_min_blocks
                            : (p.flags & (MTTS_GEMM_F_A_BF16 | MTTS_WGRAD_F_DY_BF16)) ? min_blocks16 : min_blocks) / hv;
    const int rows = batched ? b_split_rows : split_rows;
    kb *= hv;
    int s = target_blocks > 0 ? (target_blocks + tiles - 1) / tiles
                              : max((mb + tiles - 1) / tiles, (M + rows / 2) / rows);
    static const int min_steps = [] { const char *e = getenv("MTTS_WGRAD_MINSTEPS"); return e && atoi(e) > 0 ? atoi(e) : 4; }();
    s = max(1, min(s, (M + min_steps * kb - 1) / (min_steps * kb)));  // at least min_steps steps per split
    int rps = (M + s - 1) / s;
    rps = (rps + kb - 1) / kb * kb;
    *rows_per_split = max(rps, kb);
    *splits = max(1, (M + *rows_per_split - 1) / *rows_per_split);
}

extern "C" size_t mtts_conv_wgrad_workspace_size(const mtts_conv_wgrad_args *args) {
    if (!args) return 0;
    int splits, rps;
    int s2, r2;  // upper bound over every schedule (explicit targets and the default rule)
    wgrad_plan(*args, 32, kWgradMaxTarget, &splits, &rps);
    wgrad_plan(*args, 32, -1, &s2, &r2);
    splits = max(splits, s2);
    wgrad_plan(*args, 32, -1, &s2, &r2, 1, true);
    splits = max(splits, s2);
    return mtts::align_up((size_t)splits * args->N * args->K * 4, 256) + (size_t)splits * args->N * 4 + 256;
}

// mtts_wgrad_flush_cap: > 0 caps the grid of the batched weight-gradient launches (0: one workgroup per block)
std::atomic<int> g_wgrad_cap{0};

template <bool BF16, int KB, int DEPTH, bool INC, bool ABF16 = false, bool YBF16 = false, bool LIN = false, int HV = 1>
static int wgrad_launch_hv(const WgradBatch &wb, hipStream_t st) {
    using Gm = WgradGeom<BF16, KB>;
    constexpr size_t lds = Gm::kLds * HV;
    static bool attr_set = false;
    if (lds > 64 * 1024 && !attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(conv_wgrad_kernel<BF16, KB, DEPTH, INC, ABF16, YBF16, LIN, HV>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return mtts::fail(MTTS_ERR_HIP, "conv_wgrad: LDS attribute");
        attr_set = true;
    }
    const int total = wb.first[wb.njobs], cap = g_wgrad_cap.load();
    hipLaunchKernelGGL((conv_wgrad_kernel<BF16, KB, DEPTH, INC, ABF16, YBF16, LIN, HV>),
                       dim3((unsigned)(cap > 0 && cap < total ? cap : total)), dim3(kThreads * HV), lds, st, wb);
    return mtts::check_launch("conv_wgrad_kernel");
}

// MTTS_WGRAD_HV=2: the two-half workgroups for the KB = 32, one-step schedules (see conv_wgrad_kernel)
static int wgrad_hv() {
    static const int hv = [] { const char *e = getenv("MTTS_WGRAD_HV"); return e && atoi(e) == 2 ? 2 : 1; }();
    return hv;
}

template <bool BF16, int KB, int DEPTH, bool INC, bool ABF16 = false, bool YBF16 = false, bool LIN = false>
static int wgrad_launch_k(const WgradBatch &wb, bool hv2, hipStream_t st) {
    if constexpr (KB == 32 && DEPTH == 1) {
        if (hv2) return wgrad_launch_hv<BF16, KB, DEPTH, INC, ABF16, YBF16, LIN, 2>(wb, st);
    }
    return wgrad_launch_hv<BF16, KB, DEPTH, INC, ABF16, YBF16, LIN, 1>(wb, st);
}

// The linear row walk (LIN): every row's dY / A rows follow from the token row index alone.
static bool wgrad_lin_ok(const mtts_conv_wgrad_args &p) {
    static const bool off = [] { const char *e = getenv("MTTS_WGRAD_LIN"); return e && e[0] == '0'; }();
    return !off && p.in_stride == 1 && p.out_stride == 1 && p.out_off == 0 && p.To_full == p.To && p.Ti == p.To;
}

// The incremental row walk needs one wrap per step (To >= KB) and element offsets that stay inside
// int32 even for the masked rows a split walks past its end (two extra sequences of margin).
static bool wgrad_inc_ok(const mtts_conv_wgrad_args &p, int kb) {
    const int64_t ymax = ((int64_t)p.nb + 2) * p.To_full * p.ldy;
    const int64_t xmax = ((int64_t)p.nb + 2) * p.Ti * p.lda + (int64_t)(p.To + kb) * p.in_stride * p.lda;
    return p.To >= kb && ymax < (int64_t(1) << 31) && xmax < (int64_t(1) << 31) && p.out_stride >= 1 &&
           p.in_stride >= 1;
}

// Everything the instantiation choice below depends on: jobs with equal keys run the same kernel and can
// share one batched launch.
struct WgradKey {
    bool bf16, a16, y16, inc, lin, hv2;
    int kb, depth;
    bool operator==(const WgradKey &o) const {
        return bf16 == o.bf16 && a16 == o.a16 && y16 == o.y16 && inc == o.inc && lin == o.lin && hv2 == o.hv2 &&
               kb == o.kb && depth == o.depth;
    }
};

static WgradKey wgrad_key(const mtts_conv_wgrad_args &p, bool bf16, int kb, int depth, int rps) {
    WgradKey k;
    k.bf16 = bf16;
    k.kb = bf16 ? kb : 32;
    k.depth = bf16 ? depth : 1;
    k.a16 = (p.flags & MTTS_GEMM_F_A_BF16) != 0;
    k.y16 = (p.flags & MTTS_WGRAD_F_DY_BF16) != 0;
    k.inc = wgrad_inc_ok(p, k.kb);
    k.lin = k.bf16 && k.kb == 32 && k.depth == 1 && k.inc && k.a16 && !k.y16 && wgrad_lin_ok(p);
    // (any split of whole double steps is exact with two halves; the plan makes them so when hv = 2)
    k.hv2 = k.kb == 32 && k.depth == 1 && wgrad_hv() == 2 && rps % (2 * k.kb) == 0;
    return k;
}

template <bool BF16, int KB, int DEPTH>
static int wgrad_launch(const WgradBatch &wb, const WgradKey &k, hipStream_t st) {
    if constexpr (BF16 && (KB == 32 || KB == 64) && DEPTH == 1) {
        // the linear walk measured faster only with a bf16 A and an fp32 dY (19200-row conv: 44.4 vs 48.0 us;
        // fp32 / fp32 42.7 vs 42.9, bf16 dY 48.1 vs 42.9: tools/wgrad_store_ab.py) -- the staging's VALU is
        // not what bounds the other storages
        if (KB == 32 && k.lin) return wgrad_launch_k<true, 32, 1, true, true, false, true>(wb, k.hv2, st);
        if (k.a16 && k.y16)
            return k.inc ? wgrad_launch_k<true, KB, 1, true, true, true>(wb, k.hv2, st)
                         : wgrad_launch_k<true, KB, 1, false, true, true>(wb, k.hv2, st);
        if (k.y16)
            return k.inc ? wgrad_launch_k<true, KB, 1, true, false, true>(wb, k.hv2, st)
                         : wgrad_launch_k<true, KB, 1, false, false, true>(wb, k.hv2, st);
        if (k.a16)
            return k.inc ? wgrad_launch_k<true, KB, 1, true, true>(wb, k.hv2, st)
                         : wgrad_launch_k<true, KB, 1, false, true>(wb, k.hv2, st);
    }
    return k.inc ? wgrad_launch_k<BF16, KB, DEPTH, true>(wb, k.hv2, st)
                 : wgrad_launch_k<BF16, KB, DEPTH, false>(wb, k.hv2, st);
}

static int wgrad_launch_key(const WgradBatch &wb, const WgradKey &k, hipStream_t st) {
    if (!k.bf16) return wgrad_launch<false, 32, 1>(wb, k, st);
    if (k.kb == 64) return k.depth == 2 ? wgrad_launch<true, 64, 2>(wb, k, st) : wgrad_launch<true, 64, 1>(wb, k, st);
    return k.depth == 2 ? wgrad_launch<true, 32, 2>(wb, k, st) : wgrad_launch<true, 32, 1>(wb, k, st);
}

// One planned weight gradient: the kernel-side job, its instantiation key and where its slabs go.
struct WgradPlanned {
    WgradJobK k;
    WgradKey key;
    int splits;
    float *dw;
    int64_t sn, sc, sj;
    float *db;
    int accumulate;
};

// the fixed-order sums of a planned job's slabs (reduce.hip) -> dw (and db)
static int wgrad_reduce_jobs(const WgradPlanned &w, mtts_reduce_job jobs[2]) {
    const mtts_conv_wgrad_args &p = w.k.a;
    const int64_t NK = (int64_t)p.N * p.K;
    jobs[0] = mtts_reduce_job{};
    jobs[0].part = w.k.part;
    jobs[0].out = w.dw;
    jobs[0].stride = NK;
    jobs[0].n = NK;
    jobs[0].splits = w.splits;
    jobs[0].accumulate = w.accumulate;
    jobs[0].cols = p.K;
    jobs[0].cin = p.cin;
    jobs[0].sr = w.sn;
    jobs[0].sc = w.sc;
    jobs[0].sj = w.sj;
    if (!w.db) return 1;
    jobs[1] = mtts_reduce_job{};
    jobs[1].part = w.k.part_db;
    jobs[1].out = w.db;
    jobs[1].stride = p.N;
    jobs[1].n = p.N;
    jobs[1].splits = w.splits;
    jobs[1].accumulate = w.accumulate;
    return 2;
}

static int wgrad_blocks(const WgradPlanned &w) {
    const mtts_conv_wgrad_args &p = w.k.a;
    return ((p.N + 127) / 128) * ((p.K + 127) / 128) * w.splits;
}

// Deferred weight gradients (between mtts_defer_reductions(1) and the next flush, MTTS_DEFER_WGRAD != 0):
// queued here and launched batched by mtts::flush_wgrads, which mtts_flush_reductions calls first.
std::mutex g_wq_mu;
std::vector<WgradPlanned> g_wq;

static bool defer_wgrads() {
    static const bool on = [] { const char *e = getenv("MTTS_DEFER_WGRAD"); return !(e && e[0] == '0'); }();
    return on && mtts::deferring();
}

// Arrival counters of the in-kernel split sums (wgrad_combine): one zeroed pool per device, handed out as a
// ring (each launch's tiles get their own counters; the last arriver of a tile re-zeroes its counter, so a
// range is free again once its launch has run).  Opt-in, MTTS_WGRAD_FUSED_SUM=1: measured in the graph-replayed
// step (round 4, profiles/r04/fused_wgrad_sum/) the weight-gradient family took 4.2 ms instead of 1.2 + 0.29 ms
// (GEMMs + the batched reduce launches): every block's agent-scope release writes back its XCD's dirty L2
// lines (a 64 KB slab per block, ~6.5 us per 16 KB in MI355X_MICROARCH.md's price list) before its ticket, on
// the block's own critical path.  Default: the separate fixed-order reduce launch.
constexpr int kCntPool = 1 << 16;
// (A fence-free variant -- whole-line slab stores, the last arriver polling the counter with sc1 loads -- gave
// wrong sums and a poll that never matched (the counter line stale in the reader's L2): removed, round 4.)
static int32_t *wgrad_counters(int n, hipStream_t st) {
    static const bool off = [] { const char *e = getenv("MTTS_WGRAD_FUSED_SUM"); return !(e && e[0] == '1'); }();
    if (off || n <= 0 || n > kCntPool / 16) return nullptr;
    static std::mutex mu;
    static int32_t *pool[64] = {};
    static int head[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!pool[dev]) {
        // never allocated inside a stream capture (the caller then takes the separate reduce launch)
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
        int32_t *p = nullptr;
        if (hipMalloc(&p, kCntPool * sizeof(int32_t)) != hipSuccess) return nullptr;
        if (hipMemset(p, 0, kCntPool * sizeof(int32_t)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            (void)hipFree(p);
            return nullptr;
        }
        pool[dev] = p;
    }
    if (head[dev] + n > kCntPool) head[dev] = 0;
    int32_t *r = pool[dev] + head[dev];
    head[dev] += (n + 15) / 16 * 16;
    return r;
}

// mtts_wgrad_plan_mode: 0 = the batched split plan for queued gradients, the per-launch one otherwise;
// 1 / 2 = always the batched / per-launch plan (tests: a queued and an immediate gradient bitwise equal)
std::atomic<int> g_wgrad_plan_mode{0};

// rows_per_step: 32 or 64 (bf16 only), -1 = default; target_blocks: 64..1024, -1 = default;
// depth: row steps in flight, 1 or 2 (bf16 only), -1 = default
static int conv_wgrad_impl(const mtts_conv_wgrad_args *args, int32_t precision, int rows_per_step, int target_blocks,
                           int depth,
                           float *dw, int64_t sn, int64_t sc, int64_t sj, float *db, int32_t accumulate,
                           void *workspace, size_t workspace_bytes, void *hip_stream) {
    MTTS_CHECK_ARG(args != nullptr, "conv_wgrad: args is null");
    const mtts_conv_wgrad_args &p = *args;
    int rc = check_gather(p.A, p.lda, p.cin, p.ntaps, p.K);
    if (rc) return rc;
    MTTS_CHECK_ARG(p.dY && dw && p.N > 0 && p.N % 4 == 0, "conv_wgrad: null dY/dw or N % 4 != 0");
    MTTS_CHECK_ARG(p.ldy % 4 == 0 && (uintptr_t)p.dY % 16 == 0, "conv_wgrad: dY rows must be 16-byte aligned");
    MTTS_CHECK_ARG(precision == MTTS_PREC_BF16 || precision == MTTS_PREC_FP32, "conv_wgrad: bad precision");
    const bool bf16 = precision == MTTS_PREC_BF16;
    // MTTS_WGRAD_KB=64: 64-row steps by default in bf16 (A/B switch)
    static const int default_kb = [] { const char *e = getenv("MTTS_WGRAD_KB"); return e && atoi(e) == 64 ? 64 : 32; }();
    if (rows_per_step < 0) rows_per_step = bf16 ? default_kb : 32;
    if (depth < 0) depth = 1;
    if (p.flags & (MTTS_GEMM_F_A_BF16 | MTTS_WGRAD_F_DY_BF16)) {
        MTTS_CHECK_ARG(bf16 && depth == 1 && p.lda % 4 == 0 && (uintptr_t)p.A % 8 == 0,
                       "conv_wgrad: a bf16 A or dY needs bf16 precision, one step in flight and 8-byte aligned rows");
    }
    MTTS_CHECK_ARG(rows_per_step == 32 || (rows_per_step == 64 && bf16), "conv_wgrad: rows_per_step 32 (or 64 bf16)");
    MTTS_CHECK_ARG(depth == 1 || (depth == 2 && bf16), "conv_wgrad: depth 1 (or 2 bf16)");
    MTTS_CHECK_ARG(target_blocks < 0 || (target_blocks >= 64 && target_blocks <= kWgradMaxTarget),
                   "conv_wgrad: target_blocks 64..1024 (or -1)");
    if (workspace_bytes < mtts_conv_wgrad_workspace_size(args) || !workspace)
        return mtts::fail(MTTS_ERR_WORKSPACE, "conv_wgrad: workspace too small");
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    int splits, rps;
    // the two-half workgroups serve the register-staged KB = 32, one-step schedules
    const int hv = (wgrad_hv() == 2 && rows_per_step == 32 && depth == 1) ? 2 : 1;
    const bool queue = p.nb * p.To > 0 && defer_wgrads();
    const int pm = g_wgrad_plan_mode.load();
    wgrad_plan(p, rows_per_step, target_blocks, &splits, &rps, hv, pm == 1 || (pm == 0 && queue));
    WgradPlanned w;
    w.k.a = p;
    w.k.part = static_cast<float *>(workspace);
    w.k.part_db = db ? reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                                 mtts::align_up((size_t)splits * p.N * p.K * 4, 256))
                     : nullptr;
    w.k.rps = rps;
    w.k.splits = splits;
    w.k.cnt = nullptr;
    w.k.dw = dw;
    w.k.db = db;
    w.k.sn = sn;
    w.k.sc = sc;
    w.k.sj = sj;
    w.k.accumulate = accumulate;
    w.k.pad_ = 0;
    w.key = wgrad_key(p, bf16, rows_per_step, depth, rps);
    w.splits = splits;
    w.dw = dw;
    w.sn = sn;
    w.sc = sc;
    w.sj = sj;
    w.db = db;
    w.accumulate = accumulate;
    const int M = p.nb * p.To;
    if (M == 0) {
        float *part_db = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                                   mtts::align_up((size_t)splits * p.N * p.K * 4, 256));
        if (hipMemsetAsync(w.k.part, 0, (size_t)p.N * p.K * 4, st) != hipSuccess ||
            hipMemsetAsync(part_db, 0, (size_t)p.N * 4, st) != hipSuccess)
            return mtts::fail(MTTS_ERR_HIP, "conv_wgrad: memset failed");
        w.splits = 1;
        w.k.part_db = db ? part_db : nullptr;
    } else {
        // in-kernel split sums (no reduce job) when enabled and the counter pool is available
        w.k.cnt = wgrad_counters(((p.N + 127) / 128) * ((p.K + 127) / 128), st);
        if (queue) {
            std::lock_guard<std::mutex> lk(g_wq_mu);
            g_wq.push_back(w);
            return MTTS_OK;
        }
        WgradBatch wb;
        wb.job[0] = w.k;
        wb.first[0] = 0;
        wb.first[1] = wgrad_blocks(w);
        wb.njobs = 1;
        if ((rc = wgrad_launch_key(wb, w.key, st))) return rc;
        if (w.k.cnt) return MTTS_OK;
    }
    // sum of the split slabs (reduce.hip: now, or queued for the step's batched launch)
    mtts_reduce_job jobs[2];
    const int nj = wgrad_reduce_jobs(w, jobs);
    return mtts::submit_reductions(jobs, nj, st);
}

namespace mtts {
// The queued weight gradients, batched by instantiation (queue order kept within a batch), then their
// slab sums appended to the reduction queue (mtts_flush_reductions launches that right after).
int flush_wgrads(hipStream_t st) {
    std::vector<WgradPlanned> q;
    {
        std::lock_guard<std::mutex> lk(g_wq_mu);
        q.swap(g_wq);
    }
    std::vector<char> done(q.size(), 0);
    for (size_t i = 0; i < q.size(); ++i) {
        if (done[i]) continue;
        WgradBatch wb;
        wb.njobs = 0;
        wb.first[0] = 0;
        for (size_t j = i; j < q.size(); ++j) {
            if (done[j] || !(q[j].key == q[i].key)) continue;
            done[j] = 1;
            wb.job[wb.njobs] = q[j].k;
            wb.first[wb.njobs + 1] = wb.first[wb.njobs] + wgrad_blocks(q[j]);
            if (++wb.njobs == kWgradBatch) {
                if (int rc = wgrad_launch_key(wb, q[i].key, st)) return rc;
                wb.njobs = 0;
            }
        }
        if (wb.njobs > 0)
            if (int rc = wgrad_launch_key(wb, q[i].key, st)) return rc;
    }
    std::vector<mtts_reduce_job> jobs;
    for (const WgradPlanned &w : q) {
        if (w.k.cnt) continue;  // summed in-kernel
        mtts_reduce_job j2[2];
        const int n = wgrad_reduce_jobs(w, j2);
        jobs.insert(jobs.end(), j2, j2 + n);
    }
    return queue_reductions(jobs.data(), (int)jobs.size());
}

int pending_wgrad_sums() {
    std::lock_guard<std::mutex> lk(g_wq_mu);
    int n = 0;
    for (const WgradPlanned &w : g_wq) n += w.db ? 2 : 1;
    return n;
}

void discard_wgrads() {
    std::lock_guard<std::mutex> lk(g_wq_mu);
    g_wq.clear();
}
}  // namespace mtts

extern "C" void mtts_wgrad_flush_cap(int32_t blocks) { g_wgrad_cap.store(blocks > 0 ? blocks : 0); }

extern "C" void mtts_wgrad_plan_mode(int32_t mode) { g_wgrad_plan_mode.store(mode >= 0 && mode <= 2 ? mode : 0); }

extern "C" int mtts_conv_wgrad(const mtts_conv_wgrad_args *args, int32_t precision, float *dw, int64_t sn,
                               int64_t sc, int64_t sj, float *db, int32_t accumulate, void *workspace,
                               size_t workspace_bytes, void *hip_stream) {
    return conv_wgrad_impl(args, precision, -1, -1, -1, dw, sn, sc, sj, db, accumulate, workspace, workspace_bytes,
                           hip_stream);
}

extern "C" int mtts_conv_wgrad_tile(const mtts_conv_wgrad_args *args, int32_t precision, int32_t rows_per_step,
                                    int32_t target_blocks, int32_t depth, float *dw, int64_t sn, int64_t sc, int64_t sj,
                                    float *db, int32_t accumulate, void *workspace, size_t workspace_bytes,
                                    void *hip_stream) {
    return conv_wgrad_impl(args, precision, rows_per_step, target_blocks, depth, dw, sn, sc, sj, db, accumulate,
                           workspace, workspace_bytes, hip_stream);
}
