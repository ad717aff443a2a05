// Weight-gradient GEMM with LDS-DMA staging (gfx950): an OPT-IN bf16-precision schedule of mtts_conv_wgrad
// (MTTS_WGRAD_GLDS=1) for fp32 operands -- measured slower than the register-staged kernel on every step
// shape (see the launcher in conv_gemm.hip and DESIGN.md); kept as the tested base for bf16-stored operands (include/mtts_decoder.h; same contract as conv_wgrad_kernel in
// conv_gemm.hip):  part[split][n][k] = sum over the split's token rows of dY[row][n] * A_gathered[row][k].
//
// Hypothesis tested: the register-staged wgrad keeps ONE 32-row step of loads in flight per workgroup and
// its grid is about one workgroup per CU, so every step would wait a full L2/HBM round trip for 256
// cycles of MFMA work.  Result: it is not latency but per-CU bandwidth that binds (fp32 operands from
// the MALL at ~25-40 GB/s per CU); three steps in flight did not help.  Here both operands go global -> LDS by global_load_lds_dwordx4 through a
// 4-stage ring (three 32-row steps in flight, 128 KiB), no VGPR round trip:
//   * per step and operand a 32-row x 128-column fp32 tile, 512 B per row, rows in token order; each
//     wave-instruction moves two rows (lane l: row 2q + l/32, columns 4(l%32)..+3), so a thread owns
//     four token rows per step and walks them incrementally (an add and a wrap select per row);
//   * a row past the split, a column past N / K, a tap row outside [0, Ti) or a masked input row
//     (a 0/1 a_scale, staged once per workgroup into LDS as byte flags) is DMA'd from a 16-byte zero
//     constant: the mask is applied by address selection;
//   * MFMA fragments (v_mfma_f32_32x32x16_bf16, reduction over rows) are read as 8 strided dwords per
//     lane (32 lanes = 32 consecutive columns of one row: conflict-free) and packed to bf16 once.
// The bias gradient (column sums of dY) is accumulated from the staged dY tiles by the k-tile-0
// workgroups in a fixed order; partial slabs are summed by reduce.hip as for the register kernel.
// Pipeline as conv_gemm_glds.hip: per-stage __shared__ objects, a loop unrolled by the stage count,
// counted s_waitcnt vmcnt (never 0 in the loop), LDS-only barriers, DMA as inline asm (M0 set).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "gemm_epilogue.h"
#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ uint4 g_wzero16 = {0u, 0u, 0u, 0u};  // never written: source of every masked / out-of-range chunk

constexpr int kT = 128;                 // output tile: 128 (n) x 128 (k)
constexpr int kR = 32;                  // token rows per step
constexpr int kThr = 256;               // 4 waves, 2 x 2, each 64 x 64
constexpr int kRowBytes = kT * 4;       // one fp32 tile row
constexpr int kOpBytes = kR * kRowBytes;  // 16 KiB per operand and stage
constexpr int kMaskMax = 4096;          // input rows whose 0/1 mask a workgroup stages (checked on the host)

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

__device__ __forceinline__ void glds16(const void *src, void *lds_base) {
    const uint32_t lds = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)lds_base);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(lds)
        : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__global__ __launch_bounds__(kThr) void wgrad_glds_kernel(mtts_conv_wgrad_args p, int rows_per_split,
                                                           float *__restrict__ part, float *__restrict__ part_db) {
    __shared__ __attribute__((aligned(1024))) unsigned char sY0[kOpBytes], sX0[kOpBytes];
    __shared__ __attribute__((aligned(1024))) unsigned char sY1[kOpBytes], sX1[kOpBytes];
    __shared__ __attribute__((aligned(1024))) unsigned char sY2[kOpBytes], sX2[kOpBytes];
    __shared__ __attribute__((aligned(1024))) unsigned char sY3[kOpBytes], sX3[kOpBytes];
    __shared__ uint8_t smask[kMaskMax];
    __shared__ float sdb[2][kT];
    auto ybuf = [&](auto S) -> unsigned char * {
        constexpr int s = decltype(S)::value;
        if constexpr (s == 0) return sY0;
        else if constexpr (s == 1) return sY1;
        else if constexpr (s == 2) return sY2;
        else return sY3;
    };
    auto xbuf = [&](auto S) -> unsigned char * {
        constexpr int s = decltype(S)::value;
        if constexpr (s == 0) return sX0;
        else if constexpr (s == 1) return sX1;
        else if constexpr (s == 2) return sX2;
        else return sX3;
    };

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 1, wc = wave & 1;
    const int lr = lane & 31, lh = lane >> 5;
    int n0, k0, split, ktile;
    {
        const int ntn = (p.N + kT - 1) / kT, ntk = (p.K + kT - 1) / kT;
        const int wgid = mtts::xcd_relabel(blockIdx.x, gridDim.x);
        split = wgid / (ntn * ntk);
        const int t = wgid - split * ntn * ntk;
        ktile = t / ntn;
        n0 = (t - ktile * ntn) * kT;
        k0 = ktile * kT;
    }
    const int M = p.nb * p.To;
    const int r_begin = split * rows_per_split;
    const int r_end = min(M, r_begin + rows_per_split);
    const bool do_db = ktile == 0 && part_db != nullptr;
    const float inv_to = 1.0f / (float)p.To;
    const int off0 = p.off[0], offstep = p.ntaps > 1 ? p.off[1] - p.off[0] : 0;

    // ---- this thread's column chunk (4 columns) of both operands, fixed for the whole split
    const int c4 = 4 * (lane & 31);
    const bool nok = n0 + c4 < p.N;  // N % 4 == 0: a chunk is all in or all out
    const int kcol = k0 + c4;
    const bool kok = kcol < p.K;
    const int tj = kok ? kcol / p.cin : 0;
    const int tch = kok ? kcol - tj * p.cin : 0;
    const int toff = off0 + tj * offstep;

    // ---- the 0/1 input-row mask of the rows this split can touch, as LDS byte flags
    int mlo = 0;
    if (p.a_scale && r_begin < r_end) {
        const int omin = min(off0, off0 + (p.ntaps - 1) * offstep), omax = max(off0, off0 + (p.ntaps - 1) * offstep);
        int b0, u0, b1, u1;
        mtts::divmod_fast(r_begin, p.To, inv_to, b0, u0);
        mtts::divmod_fast(r_end - 1, p.To, inv_to, b1, u1);
        mlo = b0 * p.Ti + max(0, u0 * p.in_stride + omin);
        const int mhi = b1 * p.Ti + min(p.Ti - 1, u1 * p.in_stride + omax);
        for (int t = tid; t <= mhi - mlo; t += kThr) smask[t] = p.a_scale[mlo + t] != 0.f;
    }
    __syncthreads();

    // ---- per owned row (4 per step): token row m, position u, dY element offset, A input row base
    int s_m[4], s_u[4], s_y[4], s_x[4], s_i[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rr = 2 * (i * 4 + wave) + lh;
        const int m = r_begin + rr;
        int b = 0, u = 0;
        mtts::divmod_fast(min(m, M - 1), p.To, inv_to, b, u);
        s_m[i] = m;
        s_u[i] = u;
        s_y[i] = (b * p.To_full + u * p.out_stride + p.out_off) * p.ldy;
        s_i[i] = u * p.in_stride + toff;
        s_x[i] = b * p.Ti + s_i[i];
    }
    const int y_step = kR * p.out_stride * p.ldy, y_wrap = (p.To_full - p.To * p.out_stride) * p.ldy;
    const int x_step = kR * p.in_stride, x_wrap = p.Ti - p.To * p.in_stride, i_wrap = -p.To * p.in_stride;
    const void *zero = &g_wzero16;
    const bool no_mask = p.a_scale == nullptr;
    const float *ysrc = p.dY + n0 + c4;
    const float *xsrc = p.A + tch;

    auto issue = [&](auto S) {
        unsigned char *yb = ybuf(S);
        unsigned char *xb = xbuf(S);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            // branch-free validity (bitwise ops: a short-circuit && here became a branch around the flag read)
            const bool mv = s_m[i] < r_end;
            const bool yv = mv & nok;
            bool xv = mv & kok & ((unsigned)s_i[i] < (unsigned)p.Ti);
            const uint8_t f = smask[xv ? s_x[i] - mlo : 0];  // index 0 when unused: any byte will do
            xv = xv & (no_mask | (f != 0));
            glds16(yv ? static_cast<const void *>(ysrc + (uint32_t)s_y[i]) : zero, yb + (i * 4 + wave) * 1024);
            glds16(xv ? static_cast<const void *>(xsrc + (uint32_t)s_x[i] * (uint32_t)p.lda) : zero,
                   xb + (i * 4 + wave) * 1024);
            s_m[i] += kR;
            const int u = s_u[i] + kR;
            const bool wrap = u >= p.To;  // To >= 32 (host): at most one wrap per step
            s_u[i] = wrap ? u - p.To : u;
            s_y[i] += y_step + (wrap ? y_wrap : 0);
            s_x[i] += x_step + (wrap ? x_wrap : 0);
            s_i[i] += x_step + (wrap ? i_wrap : 0);
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
    float colsum = 0.f;  // do_db: column (tid & 127), rows 16 (tid >> 7) .. +15 of every step

    auto compute = [&](auto S, auto DBc) {
        constexpr bool DB = decltype(DBc)::value;
        const float *Ys = reinterpret_cast<const float *>(ybuf(S));
        const float *Xs = reinterpret_cast<const float *>(xbuf(S));
#pragma unroll
        for (int ks = 0; ks < kR / 16; ++ks) {
            const int r0 = ks * 16 + 8 * lh;
            bf16x8 af[2], bfr[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const float *col = Ys + r0 * kT + wr * 64 + i * 32 + lr;
                const uint4 w = make_uint4(pack2(col[0], col[kT]), pack2(col[2 * kT], col[3 * kT]),
                                           pack2(col[4 * kT], col[5 * kT]), pack2(col[6 * kT], col[7 * kT]));
                af[i] = __builtin_bit_cast(bf16x8, w);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const float *col = Xs + r0 * kT + wc * 64 + j * 32 + lr;
                const uint4 w = make_uint4(pack2(col[0], col[kT]), pack2(col[2 * kT], col[3 * kT]),
                                           pack2(col[4 * kT], col[5 * kT]), pack2(col[6 * kT], col[7 * kT]));
                bfr[j] = __builtin_bit_cast(bf16x8, w);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
        if constexpr (DB) {
            const float *col = Ys + (tid >> 7) * 16 * kT + (tid & (kT - 1));
#pragma unroll
            for (int r = 0; r < 16; ++r) colsum += col[r * kT];
        }
    };

    // whole rounds of 4 steps: the launcher sizes splits in multiples of 128 rows, so only the last split
    // runs (all-zero) steps past its end -- a loop with exits between the unrolled stages made hipcc
    // shuttle the accumulators between VGPRs and AGPRs every step
    const int nsteps = r_begin < r_end ? (r_end - r_begin + 4 * kR - 1) / (4 * kR) * 4 : 0;
    auto run = [&](auto DBc) {
        // prologue: steps 0..2 in flight
        issue(std::integral_constant<int, 0>{});
        issue(std::integral_constant<int, 1>{});
        issue(std::integral_constant<int, 2>{});
        // step s reads buffer s % 4 and refills buffer (s + 3) % 4, which step s - 1 read
        auto step = [&](auto S) {
            constexpr int cur = decltype(S)::value, nxt = (cur + 3) % 4;
            wait_vmcnt<8 * 2>();  // this wave's 8 DMAs of step s have landed (steps s+1, s+2 may fly)
            mtts::lds_barrier();  // ... everyone's, and step s-1's reads are done
            issue(std::integral_constant<int, nxt>{});
            compute(S, DBc);
        };
        for (int s = 0; s < nsteps; s += 4) {
            step(std::integral_constant<int, 0>{});
            step(std::integral_constant<int, 1>{});
            step(std::integral_constant<int, 2>{});
            step(std::integral_constant<int, 3>{});
        }
        wait_vmcnt<0>();  // no DMA may still target this workgroup's LDS when it retires
    };
    if (nsteps > 0) {
        if (do_db) run(std::true_type{});
        else run(std::false_type{});
    }

    float *slab = part + (size_t)split * p.N * p.K;
#pragma unroll
    for (int i = 0; i < 2; ++i)
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
        sdb[tid >> 7][tid & (kT - 1)] = colsum;
        __syncthreads();
        if (tid < kT && n0 + tid < p.N) part_db[(size_t)split * p.N + n0 + tid] = sdb[0][tid] + sdb[1][tid];
    }
}

}  // namespace

namespace mtts {

// Applies: fp32 operands, N % 4 == 0 (checked by the caller), To >= 32 (one wrap per step), element offsets
// inside int32, a NULL or 0/1 a_scale (MTTS_GEMM_F_BINARY_SCALE), and the mask rows of every split fit
// the workgroup's staging buffer.
bool wgrad_glds_applies(const mtts_conv_wgrad_args &p, int rows_per_split) {
    if (p.flags & (MTTS_GEMM_F_A_BF16 | MTTS_WGRAD_F_DY_BF16)) return false;
    if (p.To < kR || p.out_stride < 1 || p.in_stride < 1 || p.ntaps < 1) return false;
    if (p.a_scale && !(p.flags & MTTS_GEMM_F_BINARY_SCALE)) return false;
    const int64_t ymax = ((int64_t)p.nb + 2) * p.To_full * p.ldy;
    const int64_t xmax = ((int64_t)p.nb + 2) * p.Ti * (int64_t)p.lda + (int64_t)(p.To + 4 * kR) * p.in_stride * p.lda;
    if (ymax >= (int64_t(1) << 31) || xmax >= (int64_t(1) << 31)) return false;
    if (p.a_scale) {  // widest input-row range a split touches
        const int off0 = p.off[0], offl = p.off[p.ntaps - 1];
        const int omin = off0 < offl ? off0 : offl, omax = off0 < offl ? offl : off0;
        const int M = p.nb * p.To;
        for (int r0 = 0; r0 < M; r0 += rows_per_split) {
            const int r1 = (r0 + rows_per_split < M ? r0 + rows_per_split : M) - 1;
            const int b0 = r0 / p.To, u0 = r0 % p.To, b1 = r1 / p.To, u1 = r1 % p.To;
            const int lo = b0 * p.Ti + (u0 * p.in_stride + omin > 0 ? u0 * p.in_stride + omin : 0);
            const int hi = b1 * p.Ti + (u1 * p.in_stride + omax < p.Ti - 1 ? u1 * p.in_stride + omax : p.Ti - 1);
            if (hi - lo + 1 > kMaskMax) return false;
        }
    }
    return true;
}

int wgrad_glds_launch(const mtts_conv_wgrad_args &p, int splits, int rows_per_split, float *part, float *part_db,
                      hipStream_t st) {
    dim3 grid((unsigned)(((p.N + kT - 1) / kT) * ((p.K + kT - 1) / kT) * splits));
    hipLaunchKernelGGL(wgrad_glds_kernel, grid, dim3(kThr), 0, st, p, rows_per_split, part, part_db);
    return check_launch("wgrad_glds_kernel");
}

}  // namespace mtts
