// Persistent LDS-DMA implicit GEMM (round 5): the bf16 conv / linear GEMMs of the decoder and the text
// encoder on big tiles, one 512-thread workgroup per CU walking its tiles with ONE continuous DMA pipeline.
//
// Same contract as conv_gemm_kernel / conv_gemm_glds_kernel (include/mtts_decoder.h, mtts_conv_gemm) for
// MTTS_PREC_BF16 with whole-tap K steps (cin % BK == 0), a_scale NULL or a 0/1 row mask.  Why a third kernel:
// the LDS-DMA kernels of conv_gemm_glds.hip run one 64-row tile per workgroup, and a round-5 probe
// (tools/r5/fill_probe.hip, profiles/r05/fill/) measured what bounds them: L2 -> LDS DMA moves ~75 GB/s per CU
// for 128-byte row segments (~100-115 for contiguous 1 KiB pieces), so a 64 x 64 split-weight tile (24 KiB of
// operands per 1 MFLOP) can at best feed ~0.8 PFLOP/s of MFMA, and the kernels reached half of that: every
// workgroup paid a cold prologue (first DMAs from HBM) and an epilogue with no loads in flight, at one or two
// workgroups per CU.  Here
//   * tiles are 128 x 256 / 256 x 128 / 128 x 128 (8 waves of 64 x 64 or 32 x 64): half to a third of the
//     operand bytes per FLOP;
//   * a workgroup owns tiles g, g + G, g + 2G, ... (G = CUs) and the K-step pipeline runs straight across
//     tile boundaries: while the last K step of tile i computes, the DMAs of tile i + 1's first steps are in
//     flight, and they keep landing during tile i's epilogue;
//   * the epilogue stages each wave's 32 x 32 accumulator tiles through a private LDS image (16-byte row
//     stores, gemm_epilogue_vec) that no DMA ever targets.
// Numerics: the MFMAs of one output element run in the K order of conv_gemm_glds_kernel (K steps ascending,
// 16-wide sub-steps ascending, hi plane before lo plane per sub-step), so results equal that kernel's unsplit
// launches bit for bit (tests/test_gemm_pk_gpu.py).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "gemm_epilogue.h"
#include "lds_dma.h"
#include "conv_gemm_pk.h"
#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
using mtts::f32x16;
using mtts::u32x4;

constexpr int kMaxItems = 12;  // work items per workgroup (full tiles + stream-K pieces); the host widens the grid above
constexpr uint32_t kOob = mtts::kDmaOob;

// buffer_load_dwordx4 ... lds (mtts::bload16) whose scalar offset may be a compile-time constant: the K-step
// offsets of the unrolled prologue fold to literals, which the soffset operand does not accept
__device__ __forceinline__ void bload16c(uint32_t voff, u32x4 rsrc, uint32_t soff, uint32_t lds) {
    soff = __builtin_amdgcn_readfirstlane(soff);
    asm volatile("" : "+s"(soff));  // an SGPR value from here on, never a folded literal
    mtts::bload16(voff, rsrc, soff, lds);
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

// Work plan of one launch (host-computed): tiles numbered N-fastest; the first t_dp tiles (whole rounds of the
// grid) run data-parallel, one whole tile per item; the K steps of the remaining tiles (usk units) are dealt to
// the G workgroups in equal contiguous ranges (stream-K).  A tile cut by a range boundary is computed in
// segments: segment j writes its raw fp32 accumulators to slab r * pmax + j of `part` and pk_fixup_kernel sums
// the segments in order (deterministic) and runs the epilogue.
struct PkPlan {
    int tiles_n, ntiles, t_dp, nk, usk, pmax;
    float *part;
};

template <int BM, int BN, int BK, int S, bool ABF16, int NPL, int WM, int NW>
struct PkGeom {
    static constexpr int NT = 64 * NW, WN = NW / WM;
    static constexpr int TM = BM / (32 * WM), TN = BN / (32 * WN);
    // NPL = 0: exact fp32 (fp32 A and W, v_mfma_f32_32x32x2f32: the 32-true / parity-policy encoder GEMMs)
    static constexpr bool F32 = NPL == 0;
    static constexpr int ES = ABF16 ? 2 : 4, WES = F32 ? 4 : 2, NPLW = F32 ? 1 : NPL;
    static constexpr int AROW = BK * ES, WROW = BK * WES;        // bytes of one row of one K step
    static constexpr int ACPR = AROW / 16, WCPR = WROW / 16;      // 16-byte chunks per row
    static constexpr int A_BYTES = BM * AROW, W_BYTES = NPLW * BN * WROW;
    static constexpr int STAGE = A_BYTES + W_BYTES;
    static constexpr int A_INS = A_BYTES / 1024, INS = STAGE / 1024;  // 1 KiB wave-instructions per stage
    static constexpr int HI = (INS + NW - 1) / NW, LO = INS / NW, REM = INS % NW;
    static constexpr int LDS = S * STAGE + NW * 4096 + kMaxItems * BM;
    static_assert(TM >= 1 && TN >= 1 && TM * 32 * WM == BM && TN * 32 * WN == BN, "tile / wave grid");
    static_assert(A_BYTES % 1024 == 0 && STAGE % 1024 == 0, "stage must be whole 1 KiB DMA pieces");
};

// XOR swizzle of 16-byte chunk c in image row r (rows of CPR chunks; 256 / (16 CPR) rows share a 256-byte
// bank row): the 16-lane groups of a ds_read_b128 fragment read hit 16 distinct chunk slots
template <int CPR>
__device__ __forceinline__ int swz(int r) {
    return (r / (16 / CPR)) % CPR;
}

// Stream-K range boundaries b_h = floor(h * usk / G), h = 1 .. G-1 (32-bit: usk * G < 2^31, checked on the host):
// how many are < x, and how many are <= x (b_h < x <=> h * usk < x * G)
__device__ __forceinline__ int pk_cnt_lt(int x, int usk, int G) {
    return min(G - 1, max(0, (x * G + usk - 1) / usk - 1));
}
__device__ __forceinline__ int pk_cnt_le(int x, int usk, int G) { return pk_cnt_lt(x + 1, usk, G); }

// Item ii of workgroup g: (tile, first K step, end K step, slab slot or -1 for a whole tile)
struct PkItem {
    int tile, kb, ke, slot;
};
__device__ __forceinline__ PkItem pk_item(const PkPlan &pl, int g, int G, int n_dp, int ua, int ub, int ii) {
    if (ii < n_dp) return {g + ii * G, 0, pl.nk, -1};
    const int r = ua / pl.nk + (ii - n_dp);  // stream-K tile (relative to t_dp)
    const int t0 = r * pl.nk;
    const int kb = max(ua, t0) - t0, ke = min(ub, t0 + pl.nk) - t0;
    int slot = -1;
    if (kb > 0 || ke < pl.nk)  // segment index: boundaries inside (t0, t0 + kb]
        slot = r * pl.pmax + pk_cnt_le(t0 + kb, pl.usk, G) - pk_cnt_le(t0, pl.usk, G);
    return {pl.t_dp + r, kb, ke, slot};
}

template <int BM, int BN, int BK, int S, bool ABF16, int NPL, int WM, int NW>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void conv_gemm_pk_kernel(mtts_conv_gemm_args p, PkPlan pl) {
    using G = PkGeom<BM, BN, BK, S, ABF16, NPL, WM, NW>;
    constexpr int NT = G::NT, WN = G::WN, TM = G::TM, TN = G::TN, ES = G::ES, KSUB = BK / 16;
    // the S stage buffers in one array indexed at run time: the DMAs are inline asm, which hipcc's waitcnt pass
    // does not see, so no fragment read waits for them (ordering: the counted vmcnt + barrier below); the loop
    // is not unrolled by stage and the epilogue is emitted once
    __shared__ __attribute__((aligned(1024))) unsigned char sst[S * G::STAGE];
    __shared__ __attribute__((aligned(16))) float sepi[NW * 1024];  // per-wave epilogue images (never DMA'd)
    __shared__ uint8_t s_ok[kMaxItems * BM];
    auto sbuf = [&](int s) -> unsigned char * { return sst + s * G::STAGE; };

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave / WN, wc = wave % WN;
    const int lr = lane & 31, lh = lane >> 5;
    const int M = p.nb * p.To;
    const int nk = pl.nk;
    const int G_ = gridDim.x;
    const int g = mtts::xcd_relabel(blockIdx.x, G_);  // consecutive work on one XCD
    const int n_dp = pl.t_dp / G_;
    const int ua = g * pl.usk / G_, ub = (g + 1) * pl.usk / G_;  // this workgroup's stream-K units
    const int n_items = n_dp + (ub > ua ? (ub - 1) / nk - ua / nk + 1 : 0);

    const float inv_to = 1.0f / (float)p.To;
    const int off0 = p.off[0], offstep = p.ntaps > 1 ? p.off[1] - p.off[0] : 0;
    const int tapstride = offstep * p.lda;
    const u32x4 rsa = mtts::make_rsrc(p.A, (uint32_t)((long long)p.nb * p.Ti * p.lda * ES));
    const u32x4 rsw = mtts::make_rsrc(p.W, (uint32_t)((long long)G::NPLW * p.N * p.Kp * G::WES));
    const size_t w_plane = (size_t)p.N * p.Kp;

    // ---- valid-tap bits of every A row of every item, computed once up front (the only reads of a_scale: none
    // may happen while DMAs fly -- hipcc would drain them with vmcnt(0))
    for (int idx = tid; idx < n_items * BM; idx += NT) {
        const int ii = idx / BM, r = idx - ii * BM;
        const PkItem it = pk_item(pl, g, G_, n_dp, ua, ub, ii);
        const int m = it.tile / pl.tiles_n * BM + r;
        uint32_t ok = 0;
        if (m < M) {
            int b, u;
            mtts::divmod_fast(m, p.To, inv_to, b, u);
            for (int j = 0; j < p.ntaps; ++j) {
                const int irow = u * p.in_stride + off0 + j * offstep;
                bool v = irow >= 0 && irow < p.Ti;
                if (v && p.a_scale) v = p.a_scale[(size_t)b * p.Ti + irow] != 0.f;
                ok |= (uint32_t)v << j;
            }
        }
        s_ok[idx] = (uint8_t)ok;
    }
    __syncthreads();

    // ---- loader: wave w issues the stage's 1 KiB pieces q = w, w + NW, ...; piece q < A_INS is A rows, the
    // rest the W image (NPL planes of BN rows).  Per-lane state of the item being loaded:
    //   A piece: l_row = element offset of the lane's chunk in tap 0 of its source row, l_ok = valid-tap bits
    //   W piece: l_w = byte offset of the lane's chunk at K step 0 (kOob past N)
    int l_row[G::HI];
    uint32_t l_ok[G::HI], l_w[G::HI];
    int li = 0, lk = 0, lke = 0;  // item being loaded, next K step, its end
    auto load_item = [&](int ii) {  // ii >= n_items: everything OOB (DMAs past the end land zeros, unused)
        const bool tv = ii < n_items;
        const PkItem it = tv ? pk_item(pl, g, G_, n_dp, ua, ub, ii) : PkItem{0, 0, nk, -1};
        const int mt = it.tile / pl.tiles_n, m0 = mt * BM, n0 = (it.tile - mt * pl.tiles_n) * BN;
        lk = it.kb;
        lke = it.ke;
#pragma unroll
        for (int i = 0; i < G::HI; ++i) {
            const int q = i * NW + wave;
            l_row[i] = 0;
            l_ok[i] = 0;
            l_w[i] = kOob;
            if (q < G::A_INS) {
                constexpr int RPI = 1024 / G::AROW;  // rows per piece
                const int r = q * RPI + lane / G::ACPR;
                const int c = (lane % G::ACPR) ^ swz<G::ACPR>(r);
                int b = 0, u = 0;
                mtts::divmod_fast(tv && m0 + r < M ? m0 + r : 0, p.To, inv_to, b, u);
                l_ok[i] = tv ? s_ok[ii * BM + r] : 0u;
                l_row[i] = (b * p.Ti + u * p.in_stride + off0) * p.lda + c * (16 / ES);
            } else if (q < G::INS) {
                constexpr int RPI = 1024 / G::WROW;
                const int ni = (q - G::A_INS) * RPI + lane / G::WCPR;  // row of the W image
                const int pn = NPL > 1 ? ni / BN : 0;
                const int n = ni - pn * BN;
                const int c = (lane % G::WCPR) ^ swz<G::WCPR>(ni);
                if (tv && n0 + n < p.N)
                    l_w[i] = (uint32_t)((pn * w_plane + (size_t)(n0 + n) * p.Kp + c * (16 / G::WES)) * G::WES);
            }
        }
    };
    load_item(0);
    auto issue = [&](int SI) {
        const uint32_t base = mtts::lds_addr(sbuf(SI));
        const int kel = lk * BK;
        const int tap = kel / p.cin, ch = kel - tap * p.cin;
        const uint32_t soa = (uint32_t)(ch * ES), sow = (uint32_t)(kel * G::WES);
#pragma unroll
        for (int i = 0; i < G::HI; ++i) {
            const int q = i * NW + wave;
            if (q < G::A_INS) {
                const uint32_t vo = ((l_ok[i] >> min(tap, 31)) & 1u) ? (uint32_t)((l_row[i] + tap * tapstride) * ES) : kOob;
                bload16c(vo, rsa, soa, __builtin_amdgcn_readfirstlane(base + q * 1024));
            } else if (q < G::INS) {
                bload16c(l_w[i], rsw, sow, __builtin_amdgcn_readfirstlane(base + q * 1024));
            }
        }
        if (++lk == lke) load_item(++li);
    };

    f32x16 acc[TM][TN];
    auto zero_acc = [&] {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
    };
    zero_acc();

    auto compute = [&](int SI) {
        const unsigned char *sa = sbuf(SI);
        const unsigned char *sw = sa + G::A_BYTES;
        if constexpr (G::F32) {  // k = 2 kk + lh per MFMA, kk ascending: conv_gemm_kernel's fp32 order
#pragma unroll
            for (int kk = 0; kk < BK / 2; ++kk) {
                const int k = 2 * kk + lh, c = k >> 2, e = (k & 3) * 4;
                float af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int r = wr * 32 * TM + i * 32 + lr;
                    af[i] = *reinterpret_cast<const float *>(sa + r * G::AROW + ((c ^ swz<G::ACPR>(r)) << 4) + e);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = wc * 32 * TN + j * 32 + lr;
                    bfr[j] = *reinterpret_cast<const float *>(sw + n * G::WROW + ((c ^ swz<G::WCPR>(n)) << 4) + e);
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
            return;
        }
#pragma unroll
        for (int ks = 0; ks < KSUB; ++ks) {
            bf16x8 af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int r = wr * 32 * TM + i * 32 + lr;
                if constexpr (ABF16) {
                    const int c = 2 * ks + lh;
                    af[i] = *reinterpret_cast<const bf16x8 *>(sa + r * G::AROW + ((c ^ swz<G::ACPR>(r)) << 4));
                } else {
                    const int c = 4 * ks + 2 * lh;
                    const float4 x0 = *reinterpret_cast<const float4 *>(sa + r * G::AROW + ((c ^ swz<G::ACPR>(r)) << 4));
                    const float4 x1 =
                        *reinterpret_cast<const float4 *>(sa + r * G::AROW + (((c + 1) ^ swz<G::ACPR>(r)) << 4));
                    af[i] = __builtin_bit_cast(
                        bf16x8, make_uint4(pack2(x0.x, x0.y), pack2(x0.z, x0.w), pack2(x1.x, x1.y), pack2(x1.z, x1.w)));
                }
            }
#pragma unroll
            for (int pn = 0; pn < G::NPLW; ++pn) {
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = pn * BN + wc * 32 * TN + j * 32 + lr;
                    const int c = 2 * ks + lh;
                    bfr[j] = *reinterpret_cast<const bf16x8 *>(sw + n * G::WROW + ((c ^ swz<G::WCPR>(n)) << 4));
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        }
    };

    int ci = 0;
    PkItem cit = pk_item(pl, g, G_, n_dp, ua, ub, 0);
    int ck = cit.kb;
    auto finish_unit = [&] {
        if (++ck < cit.ke) return;
        const int mt = cit.tile / pl.tiles_n, m0 = mt * BM, n0 = (cit.tile - mt * pl.tiles_n) * BN;
        float *stage = sepi + wave * 1024;
        if (cit.slot < 0) {
            mtts::gemm_epilogue_vec<TM, TN>(p, acc, stage, m0 + wr * 32 * TM, n0 + wc * 32 * TN, lane);
        } else {  // raw partial tile into its slab (tile-local rows of BN floats), through the wave's LDS image
            float *slab = pl.part + (size_t)cit.slot * BM * BN;
            const int rsub = lane >> 3, c4 = lane & 7;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
#pragma unroll
                    for (int v = 0; v < 16; ++v) stage[((v & 3) + 8 * (v >> 2) + 4 * lh) * 32 + lr] = acc[i][j][v];
#pragma unroll
                    for (int it = 0; it < 4; ++it) {
                        const float4 x = reinterpret_cast<const float4 *>(stage)[(it * 8 + rsub) * 8 + c4];
                        const int row = wr * 32 * TM + i * 32 + it * 8 + rsub, col = wc * 32 * TN + j * 32 + 4 * c4;
                        *reinterpret_cast<float4 *>(slab + (size_t)row * BN + col) = x;
                    }
                }
        }
        zero_acc();
        if (++ci < n_items) {
            cit = pk_item(pl, g, G_, n_dp, ua, ub, ci);
            ck = cit.kb;
        }
    };

    const int units = n_dp * nk + (ub - ua);
    // prologue: units 0 .. S-2 in flight
    for (int s0 = 0; s0 < S - 1; ++s0) issue(s0);
    // unit v computes from buffer v % S and refills buffer (v + S - 1) % S (read by unit v - 1)
    int cur = 0;
    for (int v = 0; v < units; ++v) {
        // this wave's DMAs for unit v have landed (S - 2 younger units may still fly) ...
        if (G::REM == 0 || wave < G::REM) mtts::wait_vmcnt<G::HI * (S - 2)>();
        else mtts::wait_vmcnt<G::LO * (S - 2)>();
        mtts::lds_barrier();  // ... and everyone's; every wave is past unit v - 1's fragment reads
        issue(cur == 0 ? S - 1 : cur - 1);
        compute(cur);
        finish_unit();
        cur = cur == S - 1 ? 0 : cur + 1;
    }
    mtts::wait_vmcnt<0>();  // no DMA may still target this workgroup's LDS when it retires
}

// Sums the stream-K segments of every cut tile in segment order and runs the epilogue (float4 columns).
template <int BM, int BN>
__global__ __launch_bounds__(256) void pk_fixup_kernel(mtts_conv_gemm_args p, PkPlan pl, int G) {
    const int r = blockIdx.y;  // stream-K tile
    // segments of tile r = 1 + range boundaries strictly inside (r nk, (r + 1) nk)
    const int nseg = 1 + pk_cnt_lt((r + 1) * pl.nk, pl.usk, G) - pk_cnt_le(r * pl.nk, pl.usk, G);
    if (nseg == 1) return;  // whole tile: its workgroup ran the epilogue
    const int e = blockIdx.x * 256 + threadIdx.x;  // float4 index within the tile
    if (e >= BM * BN / 4) return;
    const int row = e / (BN / 4), col = (e - row * (BN / 4)) * 4;
    const int tile = pl.t_dp + r, mt = tile / pl.tiles_n;
    const int m = mt * BM + row, n = (tile - mt * pl.tiles_n) * BN + col;
    const int M = p.nb * p.To;
    if (m >= M || n >= p.N) return;
    const float *slab = pl.part + (size_t)r * pl.pmax * BM * BN + (size_t)row * BN + col;
    float4 a = *reinterpret_cast<const float4 *>(slab);
    for (int j = 1; j < nseg; ++j) {
        const float4 b = *reinterpret_cast<const float4 *>(slab + (size_t)j * BM * BN);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float4 bn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.bias) bn = *reinterpret_cast<const float4 *>(p.bias + n);
    float v[4] = {a.x + bn.x, a.y + bn.y, a.z + bn.z, a.w + bn.w};
    int b, u;
    mtts::divmod_fast(m, p.To, 1.0f / (float)p.To, b, u);
    uint32_t s0 = 0, s1 = 0;
    float keep = 1.f;
    if (p.dropout_p > 0.f) {
        s0 = p.seed[0];
        s1 = p.seed[1];
        keep = 1.0f / (1.0f - p.dropout_p);
    }
    mtts::epilogue_row4(p, b * p.To_full + u * p.out_stride + p.out_off, n, v, s0, s1, keep);
}

struct PkCfg {
    int bm, bn, bk, s, wm, nw;
};
// schedule ids MTTS_GEMM_PK + i
constexpr PkCfg kPk[] = {
    {128, 256, 32, 3, 2, 8},  // 0: 8 waves of 64 x 64
    {128, 128, 32, 4, 2, 8},  // 1: 8 waves of 64 x 32
    {256, 128, 32, 3, 4, 8},  // 2: 8 waves of 64 x 64
    {128, 128, 64, 2, 2, 8},  // 3: 64-wide K steps, 2 stages
    {64, 256, 32, 4, 2, 8},   // 4: 8 waves of 32 x 64
    {128, 256, 64, 2, 2, 8},  // 5: 64-wide K steps (one plane only)
    {128, 128, 32, 2, 2, 4},  // 6: 4 waves of 64 x 64, two workgroups per CU
    {64, 128, 32, 3, 2, 4},   // 7: 4 waves of 32 x 64, two per CU
    {128, 64, 32, 3, 2, 4},   // 8: 4 waves of 64 x 32, two per CU
    {64, 256, 32, 2, 1, 4},   // 9: 4 waves of 64 x 64 (one plane: two per CU)
    {64, 64, 32, 3, 2, 4},    // 10: 4 waves of 32 x 32, two per CU (exact fp32: the MFMA, not the operands, binds)
    {64, 64, 32, 2, 2, 4},    // 11: the same, two stages (three per CU)
    {32, 128, 32, 3, 1, 4},   // 12: 4 waves of 32 x 32 in a row
    {64, 64, 64, 3, 2, 4},    // 13: 64-wide K steps (128-byte bf16 row pieces), 4 waves of 32 x 32
    {64, 64, 64, 2, 2, 4},    // 14: the same, two stages
    {64, 128, 64, 2, 2, 4},   // 15: 4 waves of 32 x 64
    {128, 64, 64, 2, 2, 4},   // 16: 4 waves of 64 x 32
};
constexpr int kNumPk = sizeof(kPk) / sizeof(kPk[0]);

template <int C, bool ABF16, int NPL>
using PkG = PkGeom<kPk[C].bm, kPk[C].bn, kPk[C].bk, kPk[C].s, ABF16, NPL, kPk[C].wm, kPk[C].nw>;

template <int C, bool ABF16, int NPL>
constexpr bool pk_fits() {
    return PkG<C, ABF16, NPL>::LDS <= 160 * 1024;
}

int pk_num_cus() {
    static const int n = [] {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) {
            hipDeviceProp_t pr;
            if (hipGetDeviceProperties(&pr, dev) == hipSuccess && pr.multiProcessorCount > 0) cus = pr.multiProcessorCount;
        }
        return cus;
    }();
    return n;
}

// The launch's grid and work split.  Whole rounds of tiles run data-parallel; the rest is stream-K when every
// workgroup then gets >= 2 K steps and a workspace holds the slabs (otherwise those tiles run whole too).
template <int C, bool ABF16, int NPL>
PkPlan pk_plan(const mtts_conv_gemm_args &p, int M, size_t ws_bytes, void *ws, int *grid, size_t *need) {
    constexpr PkCfg c = kPk[C];
    using G = PkG<C, ABF16, NPL>;
    const int slots_per_cu = (c.nw == 4 && G::LDS <= 80 * 1024) ? 2 : 1;
    PkPlan pl{};
    pl.tiles_n = (p.N + c.bn - 1) / c.bn;
    pl.ntiles = ((M + c.bm - 1) / c.bm) * pl.tiles_n;
    pl.nk = p.K / c.bk;
    int Gs = pk_num_cus() * slots_per_cu;
    Gs = std::max(Gs, 1);
    const int rounds = pl.ntiles / Gs;
    const int rem = pl.ntiles - rounds * Gs;
    const long long usk = (long long)rem * pl.nk;
    static const int sk_min = [] {  // MTTS_PK_SK=0: whole tiles only; =N: stream-K from N units per workgroup
        const char *e = getenv("MTTS_PK_SK");
        return e ? (atoi(e) <= 0 ? 1 << 30 : atoi(e)) : 8;
    }();
    bool sk = rem > 0 && usk >= (long long)sk_min * Gs && (usk + 1) * Gs < (1ll << 31);
    int pmax = 0;
    if (sk) {
        const int per = (int)(usk / Gs);                 // >= 2 units per workgroup
        pmax = (pl.nk + per - 1) / per + 1;
        *need = (size_t)rem * pmax * c.bm * c.bn * sizeof(float);
        if (!ws || ws_bytes < *need || (uintptr_t)ws % 16) sk = false;
    } else {
        *need = 0;
    }
    if (sk) {
        pl.t_dp = rounds * Gs;
        pl.usk = (int)usk;
        pl.pmax = pmax;
        pl.part = static_cast<float *>(ws);
        *grid = Gs;
    } else {  // every tile whole: ceil(ntiles / G) per workgroup, at most kMaxItems
        int g = std::min(pl.ntiles, Gs);
        g = std::max(g, (pl.ntiles + kMaxItems - 1) / kMaxItems);
        const int per = (pl.ntiles + g - 1) / g;
        pl.t_dp = per * g;  // per items each; tiles past ntiles have rows >= M: no loads, no stores
        pl.usk = 0;
        pl.pmax = 0;
        pl.part = nullptr;
        *grid = g;
    }
    return pl;
}

template <int C, bool ABF16, int NPL>
int launch_pk_t(const mtts_conv_gemm_args &p, int M, void *ws, size_t ws_bytes, hipStream_t st, size_t *need_out) {
    if constexpr (!pk_fits<C, ABF16, NPL>()) {
        return mtts::fail(MTTS_ERR_UNSUPPORTED, "conv_gemm: persistent schedule does not fit LDS for this operand");
    } else {
        constexpr PkCfg c = kPk[C];
        int grid = 0;
        size_t need = 0;
        const PkPlan pl = pk_plan<C, ABF16, NPL>(p, M, ws_bytes, ws, &grid, &need);
        if (need_out) {  // workspace query only
            *need_out = need;
            return MTTS_OK;
        }
        hipLaunchKernelGGL((conv_gemm_pk_kernel<c.bm, c.bn, c.bk, c.s, ABF16, NPL, c.wm, c.nw>), dim3((unsigned)grid),
                           dim3(64 * c.nw), 0, st, p, pl);
        int rc = mtts::check_launch("conv_gemm_pk_kernel");
        if (rc || pl.usk == 0) return rc;
        const int rem = pl.ntiles - pl.t_dp;
        hipLaunchKernelGGL((pk_fixup_kernel<c.bm, c.bn>), dim3((unsigned)((c.bm * c.bn / 4 + 255) / 256), (unsigned)rem),
                           dim3(256), 0, st, p, pl, grid);
        return mtts::check_launch("pk_fixup_kernel");
    }
}

template <int C>
int launch_pk(const mtts_conv_gemm_args &p, int M, void *ws, size_t ws_bytes, hipStream_t st, size_t *need, bool f32) {
    if (f32) return launch_pk_t<C, false, 0>(p, M, ws, ws_bytes, st, need);
    const bool a16 = p.flags & MTTS_GEMM_F_A_BF16, w2 = p.flags & MTTS_GEMM_F_W_SPLIT;
    if (a16) return w2 ? launch_pk_t<C, true, 2>(p, M, ws, ws_bytes, st, need) : launch_pk_t<C, true, 1>(p, M, ws, ws_bytes, st, need);
    return w2 ? launch_pk_t<C, false, 2>(p, M, ws, ws_bytes, st, need) : launch_pk_t<C, false, 1>(p, M, ws, ws_bytes, st, need);
}

template <int... I>
int launch_pk_id(int id, const mtts_conv_gemm_args &p, int M, void *ws, size_t ws_bytes, hipStream_t st, size_t *need,
                 bool f32, std::integer_sequence<int, I...>) {
    int rc = MTTS_ERR_INVALID_ARG;
    (void)((id == I ? (rc = launch_pk<I>(p, M, ws, ws_bytes, st, need, f32), true) : false) || ...);
    return rc;
}

}  // namespace

namespace mtts {

int conv_gemm_pk_num_cfgs() { return kNumPk; }

// Whether persistent schedule `id` can run this GEMM: bf16 MFMA on one or two weight planes, whole-tap K
// steps of its BK, 16-byte aligned operand rows, a 0/1 row mask or none, 32-bit byte offsets, the 16-byte
// epilogue.
bool conv_gemm_pk_applies(int id, const mtts_conv_gemm_args &p, bool f32) {
    if (id < 0 || id >= kNumPk) return false;
    if (f32 && (p.flags & (MTTS_GEMM_F_A_BF16 | MTTS_GEMM_F_W_SPLIT | MTTS_GEMM_F_C_BF16 | MTTS_GEMM_F_PRE_BF16))) return false;
    const int bk = kPk[id].bk;
    if (p.flags & (MTTS_GEMM_F_A_SPLIT | MTTS_GEMM_F_SPLIT3)) return false;
    if (p.a_scale && !(p.flags & MTTS_GEMM_F_BINARY_SCALE)) return false;
    const bool a16 = p.flags & MTTS_GEMM_F_A_BF16;
    const int es = a16 ? 2 : 4, npl = (p.flags & MTTS_GEMM_F_W_SPLIT) ? 2 : 1;
    if (p.cin % bk || p.K % bk || p.lda % (16 / es) || (uintptr_t)p.A % 16 || p.Kp % 8 || (uintptr_t)p.W % 16) return false;
    if ((long long)p.nb * p.Ti * p.lda * es >= (1ll << 31) - (1ll << 20)) return false;
    if ((long long)npl * p.N * p.Kp * (f32 ? 4 : 2) >= (1ll << 31) - (1ll << 20)) return false;
    return mtts::gemm_epilogue_vec_ok(p);
}

size_t conv_gemm_pk_workspace_bytes(int id, const mtts_conv_gemm_args &p, bool f32) {
    size_t need = 0;
    const int M = p.nb * p.To;
    if (M == 0 || !conv_gemm_pk_applies(id, p, f32)) return 0;
    launch_pk_id(id, p, M, nullptr, 0, nullptr, &need, f32, std::make_integer_sequence<int, kNumPk>{});
    return need;
}

int conv_gemm_pk_launch(int id, const mtts_conv_gemm_args &p, int M, void *ws, size_t ws_bytes, hipStream_t st, bool f32) {
    return launch_pk_id(id, p, M, ws, ws_bytes, st, nullptr, f32, std::make_integer_sequence<int, kNumPk>{});
}

}  // namespace mtts
