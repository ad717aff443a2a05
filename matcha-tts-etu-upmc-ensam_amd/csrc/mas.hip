// Monotonic Alignment Search on gfx950 (MI355X).
//
// Replaces the reference's host round trip  (matcha/utils/monotonic_align/__init__.py:40-55:
// D2H copy -> Cython DP core.pyx:16-96 under OpenMP prange core.pyx:121 -> H2D copy) with two
// stream-ordered kernels:
//
//   mas_dp_kernel<K,...>   one wave64 per utterance (the DP is a T_y-long dependency chain, so one
//                          utterance never benefits from more than one wave).  Lane l owns the K
//                          consecutive text rows x = l*K .. l*K+K-1 of the column; the x-1 neighbour
//                          of row l*K comes from lane l-1 with one DPP `wave_shr:1` (no LDS, no
//                          barrier).  The lattice streams through registers in chunks of C columns
//                          (K*C = 32 cells per lane per chunk), double-buffered so chunk k+1 is in
//                          flight while chunk k is computed; value*mask is formed on arrival.
//                          Backpointers are bit-packed per row, 32 columns per word (bit 31-j =
//                          column j of the word), in LDS when they fit and in the workspace
//                          otherwise.  The backtrack walks rows, not columns: for the current row
//                          it jumps straight to the highest diagonal bit at or below y with one
//                          s_ff1, so it costs O(t_x + t_y/32) scalar steps instead of t_y dependent
//                          loads.  Output: per-row start column (a monotone path is one contiguous
//                          run per row).
//   mas_expand_kernel      full-chip, coalesced float4 writer of the dense [B,Tx,Ty] path
//                          (12 B/cell algorithmic traffic is dominated by this write + the reads).
//
// Numerics (bit-exact with the Cython): this file is compiled with -ffp-contract=off; value*mask is
// one fp32 multiply (__init__.py:45), `best + score` one fp32 add (core.pyx:80), ties take the
// diagonal (`from_prev >= from_same or x == y`, core.pyx:73), out-of-band cells hold max_neg_val.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "mtts_base.h"

namespace {

constexpr int kWave = 64;
constexpr int kDefaultRing = 2;  // lattice chunks in the DP ring (premasked); 3 and 4 measured equal (DP is VALU-chain bound)
constexpr int kLdsBitsLimit = 48 * 1024;  // LDS bytes for backpointer words (total stays <= 64 KiB)

struct MasArgs {
    const float *value;     // [B,Tx,Ty]
    const float *mask;      // [B,Tx,Ty] or null (lengths given explicitly)
    const int32_t *t_xs;    // [B] or null (then from mask)
    const int32_t *t_ys;    // [B] or null
    int32_t *lengths;       // [B,2] (workspace or caller)
    int32_t *row_start;     // [B,Tx]
    uint32_t *bits;         // [B, nch, Txp] (global-bits mode only)
    float *dp_out;          // [B,Tx,Ty] reference-mutated lattice, or null
    int Tx, Ty, Txp, nch;
    int premasked;
    float neg;
    int tr_ld;  // > 0: `value` is the premasked lattice TRANSPOSED, [B][Ty][tr_ld] (x contiguous; tr_ld = Txp)
    int bt_bufs;  // multi-wave kernel, global-bits mode: backtrack slot buffers in LDS (2, 1; 0: walk from global)
};

// K consecutive floats at p (the text rows x0 .. x0+K-1 of one column of a transposed lattice): one wave
// instruction moves 64 * K * 4 contiguous bytes -- the row-major lattice's lane-per-row loads touched 64 lines
// per instruction and 16 bytes of each
template <int K>
__device__ __forceinline__ void load_col_rows(const float *__restrict__ p, float (&dst)[K]) {
    if constexpr (K % 4 == 0) {
#pragma unroll
        for (int q = 0; q < K / 4; ++q) {
            const float4 v = reinterpret_cast<const float4 *>(p)[q];
            dst[4 * q] = v.x;
            dst[4 * q + 1] = v.y;
            dst[4 * q + 2] = v.z;
            dst[4 * q + 3] = v.w;
        }
    } else if constexpr (K == 2) {
        const float2 v = *reinterpret_cast<const float2 *>(p);
        dst[0] = v.x;
        dst[1] = v.y;
    } else {
#pragma unroll
        for (int q = 0; q < K; ++q) dst[q] = p[q];
    }
}

__device__ __forceinline__ float dpp_wave_shr1(float src, float lane0_value) {
    // lane l <- lane l-1; lane 0 keeps lane0_value (bound_ctrl = 0 disables the write there).
    return __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, lane0_value),
                                           __builtin_bit_cast(int, src), 0x138 /*wave_shr:1*/,
                                           0xf, 0xf, false));
}

// Loads N consecutive floats of one lattice row.  Plain global loads: on ROCm 7.2 clang the
// __builtin_amdgcn_raw_buffer_load_b64/_b128 builtins lower to a single dword load and alias every
// component to element 0 (checked in the emitted IR), so the buffer-resource path is not used.
// `eoff` is clamped so a load never leaves the utterance (columns past Ty are never consumed).
template <int N, bool VEC>
__device__ __forceinline__ void load_row_segment(const float *__restrict__ base, int eoff, int last,
                                                 float (&dst)[N]) {
    if constexpr (VEC && N % 4 == 0) {
#pragma unroll
        for (int q = 0; q < N / 4; ++q) {
            const int o = min(eoff + 4 * q, last - 3);
            const float4 v = *reinterpret_cast<const float4 *>(base + o);
            dst[4 * q + 0] = v.x;
            dst[4 * q + 1] = v.y;
            dst[4 * q + 2] = v.z;
            dst[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < N; ++q) dst[q] = base[min(eoff + q, last)];
    }
}

// One cell of the DP on the transposed lattice (TR kernels: paths only, no dp_out), the same decisions as the
// select chain of the row-major kernels (core.pyx:65-80) with no compare on the column chain:
//   from_same = d == 0 ? -inf : dp      -> min(dp, +-inf)          (the x == y forced diagonal)
//   best      = diag ? from_prev : from_same, diag = from_prev >= from_same  -> max(from_prev, from_same)
//   band      = x in [y - span, y] ? v : max_neg_val               -> med3(v, lo, hi), (lo, hi) = (-inf, +inf)
//                                                                     in band, (neg, neg) outside
// max / min pick the same VALUE as the selects (they differ only in the sign of an exact zero, which no later
// comparison sees); diag is computed beside the chain for the backpointer bit.  min and max are written as med3
// against an infinity (min(a, b) = med3(a, b, -inf), max(a, b) = med3(a, b, +inf)): fminf / fmaxf under IEEE
// mode cost a canonicalising v_max_f32 x, x per operand on the chain.
__device__ __forceinline__ float cell_tr(float fp, float dp, float sc, int d, unsigned span, float neg, bool &diag) {
    const float fs = __builtin_amdgcn_fmed3f(dp, d == 0 ? -INFINITY : INFINITY, -INFINITY);
    diag = fp >= fs;
    const float v = __builtin_amdgcn_fmed3f(fp, fs, INFINITY) + sc;
    const bool band = (unsigned)d <= span;
    return __builtin_amdgcn_fmed3f(v, band ? -INFINITY : neg, band ? INFINITY : neg);
}

// R = 2 R + (fp >= fs): the backpointer bit shifted in by v_cmp + v_addc (the compiler builds it from a cndmask, an or
// and a shift per column pair)
__device__ __forceinline__ void shift_in_ge(uint32_t &R, float fp, float fs) {
    asm("v_cmp_ge_f32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc" : "+v"(R) : "v"(fp), "v"(fs) : "vcc");
}

// max(a, b) as one v_max_f32: the compiler lowers fmaxf / a med3 against +inf to a canonicalising v_max_f32 x, x per
// operand first (IEEE mode), an extra instruction on the column chain; the DP's operands are never NaN
__device__ __forceinline__ float vmax_raw(float a, float b) {
    float r;
    asm("v_max_f32_e32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

template <int K, int C, int D, bool PM, bool VEC, bool LDS_BITS, bool DP_OUT, bool TR = false>
__global__ __launch_bounds__(kWave, 1) void mas_dp_kernel(MasArgs a) {
    static_assert(!TR || (PM && !DP_OUT), "the transposed lattice is premasked, and dp_out is row-major");
    extern __shared__ uint32_t smem[];
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const int Tx = a.Tx, Ty = a.Ty, Txp = a.Txp;
    const size_t ubase = (size_t)b * Tx * Ty;
    const float neg = a.neg;

    // ---- lengths: explicit (core.pyx API) or from the mask (__init__.py:52-53) ----
    int t_x, t_y;
    if (a.t_xs) {
        t_x = a.t_xs[b];
        t_y = a.t_ys[b];
    } else {
        const float *m = a.mask + ubase;
        float sx = 0.f, sy = 0.f;
        for (int x = lane; x < Tx; x += kWave) sx += m[(size_t)x * Ty];
        for (int y = lane; y < Ty; y += kWave) sy += m[y];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            sx += __shfl_xor(sx, off);
            sy += __shfl_xor(sy, off);
        }
        t_x = (int)sx;
        t_y = (int)sy;
    }
    t_x = __builtin_amdgcn_readfirstlane(t_x);
    t_y = __builtin_amdgcn_readfirstlane(t_y);
    if (lane == 0) {
        a.lengths[2 * b] = t_x;
        a.lengths[2 * b + 1] = t_y;
    }

    int32_t *rs = reinterpret_cast<int32_t *>(smem);  // [Txp] row starts
    uint32_t *bits_l = smem + Txp;                      // [nch][Txp] (LDS mode)
    uint32_t *bits_g = a.bits + (size_t)b * a.nch * Txp;
    for (int x = lane; x < Txp; x += kWave) rs[x] = -1;

    const bool valid = t_x >= 1 && t_y >= 1 && t_x <= t_y && t_x <= Tx && t_y <= Ty;
    if (valid) {
        // ------------------------------- forward DP -------------------------------
        const int x0 = lane * K;
        const unsigned span = (unsigned)(t_y - t_x);
        int roff[K];  // element offset of each owned row (clamped into the utterance for loads)
#pragma unroll
        for (int i = 0; i < K; ++i) roff[i] = min(x0 + i, Tx - 1) * Ty;
        const int last = Tx * Ty - 1;
        const float *vbase = TR ? a.value + (size_t)b * Ty * a.tr_ld + x0 : a.value + ubase;
        const float *mbase = PM ? vbase : a.mask + ubase;

        float dp[K];
        uint32_t R[K];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            dp[i] = neg;  // core.pyx:52-53
            R[i] = 0u;
        }

        // D-deep ring of lattice chunks: chunk c+D-1 is requested while chunk c is processed, so D-1
        // chunks (K*C*(D-1) cells per lane) are in flight -- at one wave per utterance nothing else
        // hides the L2/MALL/HBM latency of the lattice stream.  Loads are unconditional (addresses are
        // clamped into the utterance) so the waitcnt bookkeeping stays exact across the ring.
        constexpr int MD = PM ? 1 : D;  // no mask registers when value is premasked
        float vbuf[D][K][C], mbuf[MD][K][C];

        auto load_chunk = [&](auto slot, int y0) {
            constexpr int sl = decltype(slot)::value;
            if constexpr (TR) {  // column-major: one K-row vector per column
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    float col[K];
                    load_col_rows<K>(vbase + (size_t)min(y0 + j, Ty - 1) * a.tr_ld, col);
#pragma unroll
                    for (int i = 0; i < K; ++i) vbuf[sl][i][j] = col[i];
                }
                return;
            }
#pragma unroll
            for (int i = 0; i < K; ++i) load_row_segment<C, VEC>(vbase, roff[i] + y0, last, vbuf[sl][i]);
            if constexpr (!PM) {
#pragma unroll
                for (int i = 0; i < K; ++i) load_row_segment<C, VEC>(mbase, roff[i] + y0, last, mbuf[sl][i]);
            }
        };

        auto flush_bits = [&](int word_idx, int shift) {
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const uint32_t w = R[i] << shift;
                if constexpr (LDS_BITS) {
                    bits_l[word_idx * Txp + x0 + i] = w;
                } else {
                    bits_g[(size_t)word_idx * Txp + x0 + i] = w;
                }
                R[i] = 0u;
            }
        };

        // Interior chunks: when every valid text row x < t_x of the chunk's columns has 1 <= y - x <= span, no cell
        // is on the forced diagonal or outside the band, so the cell is just best-of-two + score -- the same
        // operations as the full update on those cells (bit-identical values and decisions); rows >= t_x (padding
        // lanes) then compute values nothing reads.  Most columns of a long utterance are interior.
        const int hi_row = min(kWave * K, t_x) - 1;  // the last valid text row this wave owns
        auto process_chunk = [&](auto slot, int y0) {
            constexpr int sl = decltype(slot)::value;
            if (y0 > hi_row && y0 + C - 1 <= (int)span && (TR || y0 + C <= t_y)) {  // wave-uniform
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    const int y = y0 + j;
                    const float nb = dpp_wave_shr1(dp[K - 1], neg);  // y >= 1 here
                    float ndp[K];
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        float sc;
                        if constexpr (PM) sc = vbuf[sl][i][j];
                        else sc = vbuf[sl][i][j] * mbuf[sl][i][j];  // __init__.py:45
                        const float fp = i == 0 ? nb : dp[i - 1], fs = dp[i];
                        if constexpr (!DP_OUT) {  // round 6: raw max on the chain, bit by v_cmp + v_addc (off it)
                            ndp[i] = vmax_raw(fp, fs) + sc;
                            shift_in_ge(R[i], fp, fs);
                        } else {  // (the mutated lattice is compared bit for bit: keep the select's signed zeros)
                            const bool diag = fp >= fs;
                            ndp[i] = (diag ? fp : fs) + sc;
                            R[i] = (R[i] << 1) | (diag ? 1u : 0u);
                        }
                    }
#pragma unroll
                    for (int i = 0; i < K; ++i) dp[i] = ndp[i];
                    if constexpr (DP_OUT) {
#pragma unroll
                        for (int i = 0; i < K; ++i)
                            if (x0 + i < t_x) a.dp_out[ubase + (size_t)(x0 + i) * Ty + y] = ndp[i];
                    }
                    if ((y & 31) == 31) flush_bits(y >> 5, 0);
                }
                return;
            }
            if constexpr (TR) {  // every column of the chunk (those past t_y feed nothing the backtrack reads)
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    const int y = y0 + j;
                    const float nb = dpp_wave_shr1(dp[K - 1], y == 0 ? 0.0f : neg);
                    float ndp[K];
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        bool diag;
                        ndp[i] = cell_tr(i == 0 ? nb : dp[i - 1], dp[i], vbuf[sl][i][j], y - (x0 + i), span, neg, diag);
                        R[i] = (R[i] << 1) | (diag ? 1u : 0u);
                    }
#pragma unroll
                    for (int i = 0; i < K; ++i) dp[i] = ndp[i];
                    if ((y & 31) == 31) flush_bits(y >> 5, 0);
                }
                return;
            }
#pragma unroll
            for (int j = 0; j < C; ++j) {
                const int y = y0 + j;
                if (y < t_y) {
                    float s[K];
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        if constexpr (PM) s[i] = vbuf[sl][i][j];
                        else s[i] = vbuf[sl][i][j] * mbuf[sl][i][j];  // __init__.py:45
                    }
                    // x == 0 predecessor: 0 at y == 0, max_neg_val after (core.pyx:63-64)
                    const float nb = dpp_wave_shr1(dp[K - 1], y == 0 ? 0.0f : neg);
                    float ndp[K];
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        const float fp = (i == 0) ? nb : dp[i - 1];  // core.pyx:65-66
                        const int d = y - (x0 + i);
                        // core.pyx:70-73: diag = from_prev >= from_same or x == y.  The x == y case enters as
                        // from_same = -inf (fp is never NaN, so fp >= -inf holds): one compare and one select on
                        // the column chain instead of a VALU -> SALU -> VALU mask round trip (same decisions)
                        const float fs = d == 0 ? -INFINITY : dp[i];
                        const bool diag = fp >= fs;
                        const float best = diag ? fp : fs;
                        const float v = best + s[i];                 // core.pyx:80
                        ndp[i] = ((unsigned)d <= span) ? v : neg;    // band x_min..x_max, :59-62
                        R[i] = (R[i] << 1) | (diag ? 1u : 0u);
                    }
#pragma unroll
                    for (int i = 0; i < K; ++i) dp[i] = ndp[i];
                    if constexpr (DP_OUT) {
#pragma unroll
                        for (int i = 0; i < K; ++i)
                            if (x0 + i < t_x) a.dp_out[ubase + (size_t)(x0 + i) * Ty + y] = ndp[i];
                    }
                    if ((y & 31) == 31) flush_bits(y >> 5, 0);
                }
            }
        };

        const int nload = (t_y + C - 1) / C;
        static_for<0, D - 1>([&](auto sl) { load_chunk(sl, decltype(sl)::value * C); });
        for (int c0 = 0; c0 < nload; c0 += D) {
            static_for<0, D>([&](auto sl) {
                constexpr int si = decltype(sl)::value;
                const int c = c0 + si;
                if (c < nload) {
                    load_chunk(std::integral_constant<int, (si + D - 1) % D>{}, (c + D - 1) * C);
                    process_chunk(sl, c * C);
                }
            });
        }
        if constexpr (TR) {  // the columns processed: whole chunks
            const int done_cols = nload * C;
            if (done_cols & 31) flush_bits(done_cols >> 5, 32 - (done_cols & 31));
        } else if (t_y & 31) {
            flush_bits(t_y >> 5, 32 - (t_y & 31));
        }

        if constexpr (!LDS_BITS) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        if constexpr (!LDS_BITS) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

        // ------------------------------- backtrack -------------------------------
        // Row idx occupies columns [ydec, y]; ydec = the highest column <= y whose diagonal bit is
        // set, or idx itself (forced diagonal at x == y, core.pyx:91).  Registers hold one chunk of
        // words slot-major: W[r] lane l = row r*64 + l, so the row select is static per r-segment.
        // Round 6: the step's decisions are selects (the branchy first version spent ~40 scalar instructions and six
        // branches per row step -- ~20 us of the B = 32, 120 x 600 kernel), and a segment's row starts gather in lane
        // (row & 63) of rsv, written to LDS once per segment.
        int idx = t_x - 1;
        int y = t_y - 1;
        int cur_c = -1;
        uint32_t W[K];
#pragma unroll
        for (int r = 0; r < K; ++r) W[r] = 0u;
        bool done = false;
#pragma unroll
        for (int r = K - 1; r >= 0; --r) {
            int rsv = -1;
            while (!done && idx >= kWave * r) {
                // row 0 runs down to column 0 (core.pyx:89-91: idx > 0 test); on the diagonal every remaining step is
                // forced
                if (idx == 0 || idx >= y) {
                    for (int x = lane; x <= idx; x += kWave) rs[x] = x;
                    done = true;
                    break;
                }
                const int c = y >> 5;
                if (c != cur_c) {
#pragma unroll
                    for (int rr = 0; rr < K; ++rr) {
                        if constexpr (LDS_BITS) {
                            W[rr] = bits_l[c * Txp + rr * kWave + lane];
                        } else {
                            W[rr] = bits_g[(size_t)c * Txp + rr * kWave + lane];
                        }
                    }
                    cur_c = c;
                }
                const uint32_t word = (uint32_t)__builtin_amdgcn_readlane((int)W[r], idx & (kWave - 1));
                const int base = c << 5;
                // columns <= y, and >= idx (in band) when the row's diagonal lies in this word
                const uint32_t m = word & (0xFFFFFFFFu << (31 - (y - base))) &
                                   (idx >= base ? 0xFFFFFFFFu >> (idx - base) : 0xFFFFFFFFu);
                const bool found = m != 0u || idx >= base;  // else: the run continues in the previous word
                const int ydec = m ? base + 31 - __builtin_ctz(m) : idx;
                rsv = (found && lane == (idx & (kWave - 1))) ? ydec : rsv;
                y = found ? ydec - 1 : base - 1;
                idx = found ? idx - 1 : idx;
            }
            if (rsv >= 0) rs[r * kWave + lane] = rsv;
        }
    }
    __syncthreads();
    int32_t *rs_out = a.row_start + (size_t)b * Tx;
    for (int x = lane; x < Tx; x += kWave) rs_out[x] = rs[x];
}

// ------------------------------------------------------------------------------------------------
// Multi-wave forward DP for Tx > 64 (round 4): W waves per utterance, thread t = wave*64 + lane owns the
// KL text rows t*KL .. t*KL+KL-1.  A column's cells depend only on the previous column, so the waves
// split the rows and run as a pipeline skewed by one 32-column chunk: in phase p wave w processes chunk
// p - w; the x-1 neighbour of its first row is the previous wave's last row one column earlier, which
// that wave's lane 63 wrote to an LDS edge ring (kEdgeRing chunks deep) one or two phases before; a workgroup
// barrier (LDS-only) ends every phase.  Per chunk a lane flushes one backpointer word per row (the
// chunk IS one 32-column word).  Same arithmetic per cell as mas_dp_kernel (bit-exact with core.pyx);
// the chain per column shrinks from K = Tx/64 rows per lane (one wave) to KL (e.g. Tx = 512: 8 -> 1)
// at the price of one barrier per 32 columns and W - 1 fill phases.  The backtrack is mas_dp_kernel's
// (wave 0), with the next backpointer word column prefetched while the current one is walked.
// MTTS_MAS_STAMPS (the probe harness tools/r6/mas_probe.py only, never the product): block b's thread 0 writes the
// 100 MHz clock at kernel start, after the forward DP and after the backtrack to mas_probe_stamps[b][0..2]
#ifdef MTTS_MAS_STAMPS
__device__ long long mas_probe_stamps[4096 * 4];
#define MAS_STAMP(i) \
    if (threadIdx.x == 0 && blockIdx.x < 4096) mas_probe_stamps[blockIdx.x * 4 + (i)] = wall_clock64()
#else
#define MAS_STAMP(i)
#endif
// edge ring depth in chunks: with the point-to-point hand-over (TR, KL <= 2) a wave may run up to kEdgeRing - 2 chunks
// ahead of its successor, so the successor's hand-over latency leaves the chunk period once the ring is deep
// enough: at 3 slots the period was a chunk's compute + one hand-over (round 6, tools/r6/mas_probe.py)
constexpr int kEdgeRing = 6;
template <int KL, int W, bool PM, bool VEC, bool LDS_BITS, bool DP_OUT, bool TR = false>
__global__ __launch_bounds__(64 * W) void mas_dp_mw_kernel(MasArgs a) {
    MAS_STAMP(0);
    static_assert(!TR || (PM && !DP_OUT), "the transposed lattice is premasked, and dp_out is row-major");
    constexpr int CC = 32;       // columns per chunk (one backpointer word)
    constexpr int C = CC / KL;   // columns per ring sub-chunk: KL * C = 32 cells per lane
    constexpr int KB = KL * W;   // backtrack words per lane (rows per lane of wave 0's walk)
    extern __shared__ uint32_t smem[];
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int Tx = a.Tx, Ty = a.Ty, Txp = a.Txp;
    const size_t ubase = (size_t)b * Tx * Ty;
    const float neg = a.neg;

    int t_x, t_y;
    if (a.t_xs) {
        t_x = a.t_xs[b];
        t_y = a.t_ys[b];
    } else {  // every wave reduces the mask's first column / row itself (same sums, no hand-off)
        const float *m = a.mask + ubase;
        float sx = 0.f, sy = 0.f;
        for (int x = lane; x < Tx; x += kWave) sx += m[(size_t)x * Ty];
        for (int y = lane; y < Ty; y += kWave) sy += m[y];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            sx += __shfl_xor(sx, off);
            sy += __shfl_xor(sy, off);
        }
        t_x = (int)sx;
        t_y = (int)sy;
    }
    t_x = __builtin_amdgcn_readfirstlane(t_x);
    t_y = __builtin_amdgcn_readfirstlane(t_y);
    if (threadIdx.x == 0) {
        a.lengths[2 * b] = t_x;
        a.lengths[2 * b + 1] = t_y;
    }

    int32_t *rs = reinterpret_cast<int32_t *>(smem);                // [Txp] row starts
    float *edge = reinterpret_cast<float *>(smem + Txp);            // [kEdgeRing][W][CC] last-row values per column
    // TR, KL <= 2: chunks each wave has finished (its edge values written): the waves hand over through these instead
    // of a workgroup barrier per chunk (round 6: the barriers took ~35 % of the forward DP at 8 x 512 x 4096)
    __shared__ int mw_done[W];
    if (threadIdx.x < W) mw_done[threadIdx.x] = 0;
    uint32_t *bits_l = smem + Txp + kEdgeRing * W * CC;                     // [nch][Txp] (LDS mode)
    uint32_t *bits_g = a.bits + (size_t)b * a.nch * Txp;
    for (int x = threadIdx.x; x < Txp; x += 64 * W) rs[x] = -1;
    __syncthreads();  // mw_done is zero before any wave reads it

    const bool valid = t_x >= 1 && t_y >= 1 && t_x <= t_y && t_x <= Tx && t_y <= Ty;
    if (valid) {
        const int x0 = (wave * 64 + lane) * KL;
        const unsigned span = (unsigned)(t_y - t_x);
        int roff[KL];
#pragma unroll
        for (int i = 0; i < KL; ++i) roff[i] = min(x0 + i, Tx - 1) * Ty;
        const int last = Tx * Ty - 1;
        const float *vbase = TR ? a.value + (size_t)b * Ty * a.tr_ld + x0 : a.value + ubase;
        const float *mbase = PM ? vbase : a.mask + ubase;
        float dp[KL];
        uint32_t R[KL];
#pragma unroll
        for (int i = 0; i < KL; ++i) {
            dp[i] = neg;
            R[i] = 0u;
        }
        // a 3-slot ring of sub-chunks, two in flight ahead of the one being processed: at one to eight waves
        // per CU nothing else hides the lattice stream's latency (one slot ahead measured no faster than the
        // one-wave kernel)
        // (two slots with a separate mask stream: three would spill at 8 rows per lane)
        constexpr int RING = PM ? 3 : 2;
        constexpr int MD = PM ? 1 : RING;
        float vbuf[RING][KL][C], mbuf[MD][KL][C];
        // TR, KL <= 2 rows per lane: buffer loads -- the column offset a wave-uniform scalar advanced by the column
        // stride, the lane's rows a fixed vector offset, columns past Ty out of the descriptor's range (zeros: they feed
        // nothing the backtrack reads) -- one scalar add and KL loads per column; the clamped 64-bit vector address of
        // the first version took ~6 issue slots per column of the issue-bound chain.  KL >= 4: float4 global loads.
        constexpr bool TRB = TR && KL <= 2;
        const auto tr_rsrc = [&] {
            if constexpr (TRB)
                return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.value + (size_t)b * Ty * a.tr_ld), 0,
                                                         (int)((size_t)Ty * a.tr_ld * 4), 0x00020000);
            else
                return 0;
        }();
        const int tr_lane = x0 * 4, tr_ld4 = a.tr_ld * 4;
        auto load_sub = [&](auto slot, int y0) {
            constexpr int sl = decltype(slot)::value;
            if constexpr (TRB) {
                int soff = y0 * tr_ld4;
#pragma unroll
                for (int j = 0; j < C; ++j) {
#pragma unroll
                    for (int i = 0; i < KL; ++i)
                        vbuf[sl][i][j] = __builtin_bit_cast(
                            float, __builtin_amdgcn_raw_buffer_load_b32(tr_rsrc, tr_lane + 4 * i, soff, 0));
                    soff += tr_ld4;
                }
                return;
            } else if constexpr (TR) {  // column-major: one KL-row vector per column
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    float col[KL];
                    load_col_rows<KL>(vbase + (size_t)min(y0 + j, Ty - 1) * a.tr_ld, col);
#pragma unroll
                    for (int i = 0; i < KL; ++i) vbuf[sl][i][j] = col[i];
                }
                return;
            }
#pragma unroll
            for (int i = 0; i < KL; ++i) load_row_segment<C, VEC>(vbase, roff[i] + y0, last, vbuf[sl][i]);
            if constexpr (!PM) {
#pragma unroll
                for (int i = 0; i < KL; ++i) load_row_segment<C, VEC>(mbase, roff[i] + y0, last, mbuf[sl][i]);
            }
        };
        const int nchunks = (t_y + CC - 1) / CC;
        const float *ein = edge + (wave > 0 ? wave - 1 : 0) * CC;  // the previous wave's ring row
        float *eout = edge + wave * CC;
        // one chunk: KL sub-chunks of C columns from the ring slots (P * KL + s) % RING (P = c % RING), the loads
        // of the sub-chunk RING - 1 ahead issued before each one is processed
        auto chunk = [&](auto phase3, int c) {
            constexpr int P = decltype(phase3)::value;
            const int r3 = c % kEdgeRing, p3 = (c + kEdgeRing - 1) % kEdgeRing;  // this chunk's / the previous one's ring slot
            // TR: the lane-0 neighbours of the whole chunk, read once (broadcast ds_read_b128: every lane the same
            // address) -- column y needs the previous wave's last row after column y - 1 (ring slot of chunk c, or of
            // chunk c - 1 for the chunk's first column); wave 0 has none (0 before column 0, else max_neg_val)
            float nbc[TR ? CC : 1];
            float eoc[TR ? CC : 1];
            if constexpr (TR) {
                if (wave == 0) {
#pragma unroll
                    for (int j = 0; j < CC; ++j) nbc[j] = (c == 0 && j == 0) ? 0.0f : neg;
                } else {
                    const float4 *src = reinterpret_cast<const float4 *>(ein + r3 * W * CC);
#pragma unroll
                    for (int q = 0; q < CC / 4 - 1; ++q) {
                        const float4 v = src[q];
                        nbc[4 * q + 1] = v.x;
                        nbc[4 * q + 2] = v.y;
                        nbc[4 * q + 3] = v.z;
                        nbc[4 * q + 4] = v.w;
                    }
                    const float4 v = src[CC / 4 - 1];
                    nbc[CC - 3] = v.x;
                    nbc[CC - 2] = v.y;
                    nbc[CC - 1] = v.z;
                    nbc[0] = c == 0 ? neg : edge[(p3 * W) * CC + (wave - 1) * CC + CC - 1];
                }
            }
            static_for<0, KL>([&](auto sv) {
                constexpr int s = decltype(sv)::value;
                constexpr int sl = (P * KL + s) % RING;
                const int y0 = c * CC + s * C;
                load_sub(std::integral_constant<int, (sl + RING - 1) % RING>{}, y0 + (RING - 1) * C);
                // the lane-0 neighbours of this sub-chunk's columns: column y needs the previous wave's last
                // row after column y - 1 (ring slot of chunk c, or of chunk c - 1 for the chunk's first column)
                float nbl[C];
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    const int jc = s * C + j;  // column within the chunk
                    if constexpr (TR) {
                        nbl[j] = nbc[jc];
                        continue;
                    }
                    const int y = y0 + j;
                    // read unconditionally (wave 0 reads a valid slot and ignores it): selects, no branches
                    const float prev = jc == 0 ? edge[(p3 * W) * CC + (wave > 0 ? wave - 1 : 0) * CC + CC - 1]
                                               : ein[r3 * W * CC + jc - 1];
                    const float first = wave == 0 ? 0.0f : neg;  // the column-0 predecessor of the wave's first row
                    nbl[j] = y == 0 ? first : (wave == 0 ? neg : prev);
                }
                float eo[C];
                // interior sub-chunk (see mas_dp_kernel): this wave's valid rows all strictly below the diagonal and
                // inside the band for every column -> best-of-two + score
                const int lo_row = wave * 64 * KL, hi_row = min(lo_row + 64 * KL, t_x) - 1;
                const bool interior = y0 > hi_row && y0 + C - 1 - lo_row <= (int)span && (TR || y0 + C <= t_y);
                if (interior) {
#pragma unroll
                    for (int j = 0; j < C; ++j) {
                        const float nb = dpp_wave_shr1(dp[KL - 1], nbl[j]);
                        float ndp[KL];
#pragma unroll
                        for (int i = 0; i < KL; ++i) {
                            float sc;
                            if constexpr (PM) sc = vbuf[sl][i][j];
                            else sc = vbuf[sl][i][j] * mbuf[sl][i][j];  // __init__.py:45
                            const float fp = i == 0 ? nb : dp[i - 1], fs = dp[i];
                            if constexpr (TR) {
                                ndp[i] = vmax_raw(fp, fs) + sc;
                                shift_in_ge(R[i], fp, fs);
                            } else {
                                const bool diag = fp >= fs;
                                ndp[i] = (diag ? fp : fs) + sc;
                                R[i] = (R[i] << 1) | (diag ? 1u : 0u);
                            }
                        }
#pragma unroll
                        for (int i = 0; i < KL; ++i) dp[i] = ndp[i];
                        if constexpr (DP_OUT) {
#pragma unroll
                            for (int i = 0; i < KL; ++i)
                                if (x0 + i < t_x) a.dp_out[ubase + (size_t)(x0 + i) * Ty + y0 + j] = ndp[i];
                        }
                        eo[j] = dp[KL - 1];
                    }
                } else if constexpr (TR) {  // every column (whole chunks: those past t_y feed nothing the backtrack reads)
#pragma unroll
                    for (int j = 0; j < C; ++j) {
                        const float nb = dpp_wave_shr1(dp[KL - 1], nbl[j]);
                        float ndp[KL];
#pragma unroll
                        for (int i = 0; i < KL; ++i) {
                            bool diag;
                            ndp[i] = cell_tr(i == 0 ? nb : dp[i - 1], dp[i], vbuf[sl][i][j], y0 + j - (x0 + i), span, neg,
                                             diag);
                            R[i] = (R[i] << 1) | (diag ? 1u : 0u);
                        }
#pragma unroll
                        for (int i = 0; i < KL; ++i) dp[i] = ndp[i];
                        eo[j] = dp[KL - 1];
                    }
                }
#pragma unroll
                for (int j = 0; j < C && !TR && !interior; ++j) {
                    const int y = y0 + j;
                    eo[j] = neg;
                    if (y < t_y) {
                        float sc[KL];
#pragma unroll
                        for (int i = 0; i < KL; ++i) {
                            if constexpr (PM) sc[i] = vbuf[sl][i][j];
                            else sc[i] = vbuf[sl][i][j] * mbuf[sl][i][j];  // __init__.py:45
                        }
                        const float nb = dpp_wave_shr1(dp[KL - 1], nbl[j]);
                        float ndp[KL];
#pragma unroll
                        for (int i = 0; i < KL; ++i) {
                            const float fp = (i == 0) ? nb : dp[i - 1];  // core.pyx:65-66
                            const int d = y - (x0 + i);
                            const float fs = d == 0 ? -INFINITY : dp[i];  // core.pyx:70-73 (see mas_dp_kernel)
                            const bool diag = fp >= fs;
                            const float best = diag ? fp : fs;
                            const float v = best + sc[i];                // core.pyx:80
                            ndp[i] = ((unsigned)d <= span) ? v : neg;    // band, :59-62
                            R[i] = (R[i] << 1) | (diag ? 1u : 0u);
                        }
#pragma unroll
                        for (int i = 0; i < KL; ++i) dp[i] = ndp[i];
                        if constexpr (DP_OUT) {
#pragma unroll
                            for (int i = 0; i < KL; ++i)
                                if (x0 + i < t_x) a.dp_out[ubase + (size_t)(x0 + i) * Ty + y] = ndp[i];
                        }
                        eo[j] = dp[KL - 1];
                    }
                }
                if constexpr (TR) {
#pragma unroll
                    for (int j = 0; j < C; ++j) eoc[s * C + j] = eo[j];
                } else if (lane == 63) {
#pragma unroll
                    for (int j = 0; j < C; ++j) eout[r3 * W * CC + s * C + j] = eo[j];
                }
            });
            if constexpr (TR) {
                if (lane == 63) {
                    float4 *dst = reinterpret_cast<float4 *>(eout + r3 * W * CC);
#pragma unroll
                    for (int q = 0; q < CC / 4; ++q)
                        dst[q] = make_float4(eoc[4 * q], eoc[4 * q + 1], eoc[4 * q + 2], eoc[4 * q + 3]);
                }
            }
            // the chunk's backpointer word per row (a partial last chunk left-aligned like mas_dp_kernel's)
            const int sh = (!TR && c == nchunks - 1 && (t_y & 31)) ? 32 - (t_y & 31) : 0;  // TR: all 32 columns ran
#pragma unroll
            for (int i = 0; i < KL; ++i) {
                const uint32_t w = R[i] << sh;
                if constexpr (LDS_BITS) bits_l[c * Txp + x0 + i] = w;
                else bits_g[(size_t)c * Txp + x0 + i] = w;
                R[i] = 0u;
            }
        };
        static_for<0, RING - 1>([&](auto sv) { load_sub(sv, decltype(sv)::value * C); });
        // (KL >= 4 keeps the barrier: there the spinning waves measured slower -- they take issue slots from their
        // SIMD partners -- 2 x 4096 x 4200 DP 1466 -> 1581 us, 1 x 5000 x 5600 3798 -> 4058 us; KL = 1 / 2: 8 x 512 x 4096
        // 250 -> 227 us, 8 x 1024 x 4096 572 -> 497 us; tools/r6/mas_probe.py)
        if constexpr (TR && KL <= 2) {
            // point-to-point hand-over: before chunk c, wave w waits until wave w - 1 has finished chunk c (its edge
            // values for c and c - 1 are in the ring) and until wave w + 1 has finished chunk c - kEdgeRing + 1 (the last
            // reader of the ring slot chunk c overwrites: wave w + 1 reads the slot of chunk c - kEdgeRing in its chunk
            // c - kEdgeRing and that slot's last value in its next chunk); after chunk c it publishes c + 1 once its LDS
            // writes have landed.  The spin is
            // bounded (every wave reaches the end whatever happens); a bound hit would only corrupt the path.
            auto wait_ge = [&](int w2, int target) {
                for (int spins = 0; spins < (1 << 22); ++spins) {
                    if (__hip_atomic_load(&mw_done[w2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) break;
                    __builtin_amdgcn_s_sleep(1);
                }
                asm volatile("" ::: "memory");  // the ring reads stay after the wait
            };
            for (int c = 0; c < nchunks; c += RING) {
                bool go = true;
                static_for<0, RING>([&](auto pv) {
                    constexpr int P = decltype(pv)::value;
                    const int cc = c + P;
                    if (go && cc < nchunks) {
                        if (wave > 0) wait_ge(wave - 1, cc + 1);
                        if (wave < W - 1 && cc >= kEdgeRing - 1) wait_ge(wave + 1, cc - kEdgeRing + 2);
                        chunk(pv, cc);
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's edge writes have landed
                        if (lane == 0)
                            __hip_atomic_store(&mw_done[wave], cc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {
                        go = false;
                    }
                });
            }
        } else {
            for (int i = 0; i < wave; ++i) mtts::lds_barrier();  // pipeline fill: wave w starts in phase w
            for (int c = 0; c < nchunks; c += RING) {
                bool go = true;
                static_for<0, RING>([&](auto pv) {
                    constexpr int P = decltype(pv)::value;
                    if (go && c + P < nchunks) {
                        chunk(pv, c + P);
                        mtts::lds_barrier();
                    } else {
                        go = false;
                    }
                });
            }
            for (int i = wave; i < W - 1; ++i) mtts::lds_barrier();  // drain: every wave runs nchunks + W - 1 phases
        }
    }
    if constexpr (!LDS_BITS) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if constexpr (!LDS_BITS) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    MAS_STAMP(1);

    if constexpr (LDS_BITS) {
        if (valid && wave == 0) {
            // backtrack (mas_dp_kernel's walk): registers hold one word column slot-major, W[r] lane l = row r*64 + l
            int idx = t_x - 1;
            int y = t_y - 1;
            int cur_c = -1;
            uint32_t Wc[KB];
#pragma unroll
            for (int r = 0; r < KB; ++r) Wc[r] = 0u;
            bool done = false;
#pragma unroll
            for (int r = KB - 1; r >= 0; --r) {
                int rsv = -1;  // the segment's row starts, lane (row & 63); selects per step (mas_dp_kernel's walk)
                while (!done && idx >= kWave * r) {
                    if (idx == 0 || idx >= y) {
                        for (int x = lane; x <= idx; x += kWave) rs[x] = x;
                        done = true;
                        break;
                    }
                    const int c = y >> 5;
                    if (c != cur_c) {
#pragma unroll
                        for (int rr = 0; rr < KB; ++rr) Wc[rr] = bits_l[c * Txp + rr * kWave + lane];
                        cur_c = c;
                    }
                    const uint32_t word = (uint32_t)__builtin_amdgcn_readlane((int)Wc[r], idx & (kWave - 1));
                    const int base = c << 5;
                    const uint32_t m = word & (0xFFFFFFFFu << (31 - (y - base))) &
                                       (idx >= base ? 0xFFFFFFFFu >> (idx - base) : 0xFFFFFFFFu);
                    const bool found = m != 0u || idx >= base;
                    const int ydec = m ? base + 31 - __builtin_ctz(m) : idx;
                    rsv = (found && lane == (idx & (kWave - 1))) ? ydec : rsv;
                    y = found ? ydec - 1 : base - 1;
                    idx = found ? idx - 1 : idx;
                }
                if (rsv >= 0) rs[r * kWave + lane] = rsv;
            }
        }
    } else if (valid && a.bt_bufs == 0) {
        if (wave == 0) {
            // backtrack from global bits (a Ty too long for the LDS slot buffers below): lane l holds the word of row
            // 64 r + l in column cur_c, loaded when the walk enters the column (latency-bound, but registers independent
            // of KL: the round-5 walk held all KB words of a column, 2 x 128 registers at KL = 16)
            int idx = t_x - 1;
            int y = t_y - 1;
            bool done = false;
#pragma unroll 1
            for (int r = (t_x - 1) / kWave; r >= 0; --r) {
                int cur_c = -1, rsv = -1;
                uint32_t Wc = 0u;
                while (!done && idx >= kWave * r) {
                    if (idx == 0 || idx >= y) {
                        for (int x = lane; x <= idx; x += kWave) rs[x] = x;
                        done = true;
                        break;
                    }
                    const int c = y >> 5;
                    if (c != cur_c) {
                        Wc = bits_g[(size_t)c * Txp + r * kWave + lane];
                        cur_c = c;
                    }
                    const uint32_t word = (uint32_t)__builtin_amdgcn_readlane((int)Wc, idx & (kWave - 1));
                    const int base = c << 5;
                    const uint32_t m = word & (0xFFFFFFFFu << (31 - (y - base))) &
                                       (idx >= base ? 0xFFFFFFFFu >> (idx - base) : 0xFFFFFFFFu);
                    const bool found = m != 0u || idx >= base;
                    const int ydec = m ? base + 31 - __builtin_ctz(m) : idx;
                    rsv = (found && lane == (idx & (kWave - 1))) ? ydec : rsv;
                    y = found ? ydec - 1 : base - 1;
                    idx = found ? idx - 1 : idx;
                }
                if (rsv >= 0) rs[r * kWave + lane] = rsv;
            }
        }
    } else if (valid) {
        // backtrack, global-bits mode (round 6): the walk of row slot r (rows 64 r .. 64 r + 63) reads only that slot's
        // word of each column, so the slot's words of all columns are copied into LDS (nch x 256 B, coalesced) and wave 0
        // walks them from there -- with two buffers the other waves copy slot r - 1 while wave 0 walks slot r.  The
        // first version loaded all KB words of a column from HBM / L2 whenever the walk entered it, one column ahead.
        const int nbuf = a.bt_bufs;
        const int slot_words = a.nch * kWave;
        int idx = t_x - 1;
        int y = t_y - 1;
        int cur_c = -1;
        uint32_t Wc = 0u;  // lane l: the word of row 64 r + l in column cur_c (one LDS read per column change)
        bool done = false;
        const int r0 = (t_x - 1) / kWave;
        auto copy_slot = [&](int r, int t0, int nt) {
            uint32_t *dst = bits_l + (nbuf == 2 ? (r & 1) * slot_words : 0);
            for (int i = t0; i < slot_words; i += nt) dst[i] = bits_g[(size_t)(i >> 6) * Txp + r * kWave + (i & (kWave - 1))];
        };
        if (nbuf == 2) copy_slot(r0, threadIdx.x, 64 * W);
#pragma unroll 1
        for (int r = r0; r >= 0; --r) {  // block-uniform
            cur_c = -1;
            if (nbuf == 1) {
                __syncthreads();  // the previous slot's walk has finished reading the buffer
                copy_slot(r, threadIdx.x, 64 * W);
            }
            __syncthreads();  // slot r is in LDS
            const uint32_t *slot = bits_l + (nbuf == 2 ? (r & 1) * slot_words : 0);
            if (wave == 0) {
                // the slot's row starts gather in lane (row & 63) of rsv (a lane select) and go to LDS once per slot; the
                // step's decisions are selects, not branches (the first version spent ~40 scalar instructions and six
                // branches per row step).  (A read-ahead of the previous column's word, round 6, measured slower:
                // 8 x 512 x 4096 89 -> 100 us, 2 x 4096 x 4200 525 -> 653 us.)
                int rsv = -1;
                while (!done && idx >= kWave * r) {
                    if (idx == 0 || idx >= y) {  // the rest of the path is the diagonal x == y (or row 0 at column 0)
                        for (int x = lane; x <= idx; x += kWave) rs[x] = x;
                        done = true;
                        break;
                    }
                    const int c = y >> 5;
                    if (c != cur_c) {
                        Wc = slot[c * kWave + lane];
                        cur_c = c;
                    }
                    const uint32_t word = (uint32_t)__builtin_amdgcn_readlane((int)Wc, idx & (kWave - 1));
                    const int base = c << 5;
                    const uint32_t m = word & (0xFFFFFFFFu << (31 - (y - base))) &
                                       (idx >= base ? 0xFFFFFFFFu >> (idx - base) : 0xFFFFFFFFu);
                    const bool found = m != 0u || idx >= base;
                    const int ydec = m ? base + 31 - __builtin_ctz(m) : idx;
                    rsv = (found && lane == (idx & (kWave - 1))) ? ydec : rsv;
                    y = found ? ydec - 1 : base - 1;
                    idx = found ? idx - 1 : idx;
                }
                if (rsv >= 0) rs[r * kWave + lane] = rsv;
            } else if (nbuf == 2 && r > 0) {
                copy_slot(r - 1, threadIdx.x - 64, 64 * (W - 1));  // beside the walk
            }
            if (nbuf == 2) __syncthreads();  // slot r - 1 copied; slot r's buffer is free for slot r - 2
        }
    }
    __syncthreads();
    MAS_STAMP(2);
    int32_t *rs_out = a.row_start + (size_t)b * Tx;
    for (int x = threadIdx.x; x < Tx; x += 64 * W) rs_out[x] = rs[x];
}

// Dense writer: path[b,x,y] = 1 iff row_start[b,x] <= y <= row_end[b,x].  One block per (b, x,
// 1024-column slab); float4 stores when rows are 16-byte aligned.
template <typename T, bool SET_ONLY>
__global__ __launch_bounds__(256) void mas_expand_kernel(const int32_t *__restrict__ row_start,
                                                         const int32_t *__restrict__ lengths,
                                                         T *__restrict__ path, int Tx, int Ty,
                                                         int vec4) {
    const int b = blockIdx.z, x = blockIdx.y;
    const int t_x = lengths[2 * b], t_y = lengths[2 * b + 1];
    const int32_t *rsb = row_start + (size_t)b * Tx;
    int s = rsb[x];
    int e = -1;
    if (s >= 0) e = (x == t_x - 1) ? t_y - 1 : rsb[x + 1] - 1;
    if (s < 0) s = 1;  // empty range
    T *row = path + ((size_t)b * Tx + x) * Ty;
    const int y0 = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (y0 >= Ty) return;
    if constexpr (SET_ONLY) {
        for (int k = 0; k < 4 && y0 + k < Ty; ++k)
            if (y0 + k >= s && y0 + k <= e) row[y0 + k] = (T)1;
    } else {
        if (vec4 && y0 + 3 < Ty) {
            float4 v;
            v.x = (y0 + 0 >= s && y0 + 0 <= e) ? 1.f : 0.f;
            v.y = (y0 + 1 >= s && y0 + 1 <= e) ? 1.f : 0.f;
            v.z = (y0 + 2 >= s && y0 + 2 <= e) ? 1.f : 0.f;
            v.w = (y0 + 3 >= s && y0 + 3 <= e) ? 1.f : 0.f;
            *reinterpret_cast<float4 *>(row + y0) = v;
        } else {
            for (int k = 0; k < 4 && y0 + k < Ty; ++k)
                row[y0 + k] = (y0 + k >= s && y0 + k <= e) ? (T)1 : (T)0;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Fused producer: the log-prior lattice of matcha_tts.py:277-282 (MatchaTTS.forward) computed
// straight from mu_x [B,C,Tx] and y [B,C,Ty] (channel-major, as the encoder / data loader hold them)
// and multiplied by the attention mask x_mask[i] * y_mask[j] (maximum_path's value*mask,
// __init__.py:45), written once to HBM for the DP:
//   ysq[j]   = sum_c -0.5 * (y[c,j] * y[c,j])            (y_square = factor^T @ y^2)
//   ymu[i,j] = sum_c (-mu[c,i]) * y[c,j]                 (y_mu_double = (2 * factor * mu)^T @ y)
//   musq[i]  = sum_c -0.5 * (mu[c,i] * mu[c,i])          (mu_square = sum(factor * mu^2, 1))
//   lattice  = ((ysq[j] - ymu[i,j]) + musq[i]) + const,  const = -0.5 * log(2 pi) * C
// Every product and sum is one fp32 operation in ascending c (-ffp-contract=off for this file): a
// numpy restatement reproduces the lattice bit for bit (oracle/prior_oracle.py).  The reference's
// torch matmuls sum in an implementation-defined order, so lattices agree to fp32 rounding, not bits.
// Tile: 64 text rows x 64 frames per 256-thread block, 4 x 4 cells per thread, mu / y tiles staged
// in LDS 16 channels at a time.  The block of tile (0, 0) also writes t_x / t_y as int32 for the DP.
constexpr int kLpT = 64;
constexpr int kLpC = 80;  // channels staged per LDS round: all of n_feats = 80 in one (16 per round left five
                           // dependent load -> barrier -> compute rounds per block: 39 us for 32 x 120 x 600)

// TR: the lattice is written transposed, out[b][j][i] with row length LX (the DP's padded row count; rows
// Tx .. LX-1 come out 0: their mask is 0), for the DP's column-major loads.
template <bool TR>
__global__ __launch_bounds__(256) void log_prior_kernel(const float *__restrict__ mu, const float *__restrict__ y,
                                                        const int64_t *__restrict__ xl, const int64_t *__restrict__ yl,
                                                        int C, int Tx, int Ty, float cst, float *__restrict__ out,
                                                        int32_t *__restrict__ txy, int LX) {
    __shared__ __attribute__((aligned(16))) float smu[kLpC][kLpT];
    __shared__ __attribute__((aligned(16))) float sy[kLpC][kLpT];
    const int b = blockIdx.z, i0 = blockIdx.y * kLpT, j0 = blockIdx.x * kLpT;
    const int tid = threadIdx.x, ti = (tid >> 4) * 4, tj = (tid & 15) * 4;
    const int t_x = (int)min<int64_t>(max<int64_t>(xl[b], 0), Tx);
    const int t_y = (int)min<int64_t>(max<int64_t>(yl[b], 0), Ty);
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) {
        txy[b] = t_x;
        txy[gridDim.z + b] = t_y;
    }
    const float *mub = mu + (size_t)b * C * Tx, *yb = y + (size_t)b * C * Ty;
    // the squared-norm terms are per row (musq) and per frame (ysq): threads 0..63 own the tile's rows, 64..127 its
    // frames, each accumulating in channel order exactly as every thread of a row / frame used to (same values)
    __shared__ float s_musq[kLpT], s_ysq[kLpT];
    float ymu[4][4], ysq[4], musq[4], sq = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int q = 0; q < 4; ++q) ymu[r][q] = 0.f;
    }
    for (int c0 = 0; c0 < C; c0 += kLpC) {
#pragma unroll 4
        for (int e = tid; e < kLpC * kLpT; e += 256) {
            const int c = c0 + e / kLpT, t = e % kLpT;
            smu[e / kLpT][t] = (c < C && i0 + t < Tx) ? mub[(size_t)c * Tx + i0 + t] : 0.f;
            sy[e / kLpT][t] = (c < C && j0 + t < Ty) ? yb[(size_t)c * Ty + j0 + t] : 0.f;
        }
        __syncthreads();
        const int cn = min(kLpC, C - c0);
        if (tid < 2 * kLpT) {  // wave-uniform: waves 0-1 rows, waves 2-3 frames
            const float *col = tid < kLpT ? &smu[0][tid] : &sy[0][tid - kLpT];
            for (int c = 0; c < cn; ++c) {
                const float v = col[c * kLpT];
                sq = sq + -0.5f * (v * v);
            }
        }
#pragma unroll 4
        for (int c = 0; c < cn; ++c) {
            const float4 m4 = *reinterpret_cast<const float4 *>(&smu[c][ti]);
            const float4 y4 = *reinterpret_cast<const float4 *>(&sy[c][tj]);
            const float mv[4] = {m4.x, m4.y, m4.z, m4.w}, yv[4] = {y4.x, y4.y, y4.z, y4.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
                for (int q = 0; q < 4; ++q) ymu[r][q] = ymu[r][q] + (-mv[r]) * yv[q];
            }
        }
        __syncthreads();
    }
    if (tid < kLpT) s_musq[tid] = sq;
    else if (tid < 2 * kLpT) s_ysq[tid - kLpT] = sq;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        musq[r] = s_musq[ti + r];
        ysq[r] = s_ysq[tj + r];
    }
    if constexpr (TR) {
        float v[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + ti + r;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = j0 + tj + q;
                const float m = (i < t_x && j < t_y) ? 1.f : 0.f;  // x_mask[i] * y_mask[j]
                v[r][q] = (((ysq[q] - ymu[r][q]) + musq[r]) + cst) * m;
            }
        }
        // through LDS (the staging tiles are free after the last channel round's barrier): the tile's 64 frames
        // x 64 rows leave as 256-byte row segments, one frame per 16 threads
        __shared__ __attribute__((aligned(16))) float tr[32][kLpT + 4];  // half the tile's frames per pass
#pragma unroll
        for (int half = 0; half < 2; ++half) {  // frames [32 * half, 32 * half + 32) per pass
            if ((tj >> 5) == half) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    *reinterpret_cast<float4 *>(&tr[(tj & 31) + q][ti]) = make_float4(v[0][q], v[1][q], v[2][q], v[3][q]);
            }
            __syncthreads();
#pragma unroll
            for (int e = 0; e < 2; ++e) {  // 32 frames x 16 float4 = 512 float4 / 256 threads
                const int f = (tid >> 4) + 16 * e, c4 = (tid & 15) * 4;
                const int j = j0 + 32 * half + f;
                if (j < Ty)  // i0 + c4 + 3 < LX: LX is a multiple of the 64-row tile
                    *reinterpret_cast<float4 *>(out + ((size_t)b * Ty + j) * LX + i0 + c4) =
                        *reinterpret_cast<const float4 *>(&tr[f][c4]);
            }
            __syncthreads();
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = i0 + ti + r;
        if (i >= Tx) continue;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = j0 + tj + q;
            const float m = (i < t_x && j < t_y) ? 1.f : 0.f;  // x_mask[i] * y_mask[j]
            v[q] = (((ysq[q] - ymu[r][q]) + musq[r]) + cst) * m;
        }
        float *row = out + ((size_t)b * Tx + i) * Ty + j0 + tj;
        if ((Ty & 3) == 0 && j0 + tj + 3 < Ty) {
            *reinterpret_cast<float4 *>(row) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (j0 + tj + q < Ty) row[q] = v[q];
        }
    }
}

// The public maximum_path(value, mask)'s lattice, premasked and transposed for the DP's column-major
// loads: out[b][y][x] = value[b][x][y] * mask[b][x][y] (the one fp32 multiply of __init__.py:45, as the DP
// forms it on arrival), 0 for Tx <= x < LX.  64 x 64 tiles through LDS, coalesced both ways.
__global__ __launch_bounds__(256) void mas_transpose_kernel(const float *__restrict__ value,
                                                            const float *__restrict__ mask, int Tx, int Ty, int LX,
                                                            float *__restrict__ out) {
    __shared__ float t[64][65];
    const int b = blockIdx.z, x0 = blockIdx.y * 64, y0 = blockIdx.x * 64;
    const size_t ib = (size_t)b * Tx * Ty;
    const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
    for (int r = r0; r < 64; r += 4) {
        const int x = x0 + r, yy = y0 + c;
        float v = 0.f;
        if (x < Tx && yy < Ty) {
            const size_t e = ib + (size_t)x * Ty + yy;
            v = mask ? value[e] * mask[e] : value[e];
        }
        t[r][c] = v;
    }
    __syncthreads();
    for (int r = r0; r < 64; r += 4) {
        const int yy = y0 + r, x = x0 + c;
        if (yy < Ty && x < LX) out[((size_t)b * Ty + yy) * LX + x] = t[c][r];
    }
}

// Alignment consumers from the row starts (matcha_tts.py:287-288, 504-505): durations
// dur[b,x] = sum_y attn[b,x,y] (the run length of row x) and col_row[b,y] = the text row of frame y
// (-1 past t_y), which turns mu_y = attn^T mu_x into a gather.  One block per utterance.
__global__ __launch_bounds__(256) void mas_runs_kernel(const int32_t *__restrict__ row_start,
                                                       const int32_t *__restrict__ lengths, int Tx, int Ty,
                                                       float *__restrict__ dur, int32_t *__restrict__ col_row) {
    const int b = blockIdx.x;
    const int t_x = lengths[2 * b], t_y = lengths[2 * b + 1];
    const int32_t *rs = row_start + (size_t)b * Tx;
    for (int x = threadIdx.x; x < Tx; x += 256) {
        const int s = rs[x];
        int n = 0;
        if (s >= 0) n = ((x == t_x - 1) ? t_y : rs[x + 1]) - s;
        if (dur) dur[(size_t)b * Tx + x] = (float)n;
    }
    if (!col_row) return;
    const bool any = t_x >= 1 && rs[0] >= 0;
    for (int yy = threadIdx.x; yy < Ty; yy += 256) {
        int row = -1;
        if (any && yy < t_y) {  // last row whose start <= yy (starts increase along the path)
            int lo = 0, hi = t_x - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (rs[mid] <= yy) lo = mid; else hi = mid - 1;
            }
            row = lo;
        }
        col_row[(size_t)b * Ty + yy] = row;
    }
}

// mu_y[b,c,y] = mu_x[b,c,col_row[b,y]] (0 where col_row < 0): attn^T mu_x on a one-hot attn is exactly
// this gather (every other term is 0 * finite).  Backward: dmu_x[b,c,x] = sum over the run of row x
// of dmu_y[b,c,y], in ascending y (deterministic; no atomics).
__global__ __launch_bounds__(256) void expand_rows_fwd_kernel(const float *__restrict__ src,
                                                              const int32_t *__restrict__ col_row, int C, int Tx,
                                                              int Ty, float *__restrict__ dst) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    const int b = blockIdx.y;
    if (idx >= (size_t)C * Ty) return;
    const int c = (int)(idx / Ty), yy = (int)(idx - (size_t)c * Ty);
    const int x = col_row[(size_t)b * Ty + yy];
    dst[((size_t)b * C + c) * Ty + yy] = x >= 0 ? src[((size_t)b * C + c) * Tx + x] : 0.f;
}

// one block per (utterance, 2 channels): the channels' dy rows are staged in LDS (16-byte coalesced
// loads when the rows allow), then 16 lanes per (channel, row x) sum its run from LDS.  The
// earlier 8-channel blocks gave B*10 workgroups -- 80 at the long-form shape (B=8, Ty=4096), 940 us per
// call on a latency-bound load phase; 2 channels give 4x the workgroups and 16-byte loads.
constexpr int kErC = 2;
constexpr int kErMaxTy = 4096;
template <bool kVec>
__global__ __launch_bounds__(256) void expand_rows_bwd_kernel(const float *__restrict__ dy,
                                                              const int32_t *__restrict__ row_start,
                                                              const int32_t *__restrict__ lengths, int C, int Tx,
                                                              int Ty, float *__restrict__ dx) {
    __shared__ __attribute__((aligned(16))) float sdy[kErC * kErMaxTy];
    const int b = blockIdx.y, c0 = blockIdx.x * kErC;
    const int nc = min(kErC, C - c0);
    const int t_x = lengths[2 * b], t_y = lengths[2 * b + 1];
    const int32_t *rs = row_start + (size_t)b * Tx;
    for (int ty0 = 0; ty0 < Ty; ty0 += kErMaxTy) {  // frame slabs (one slab for Ty <= 4096)
        const int tn = min(kErMaxTy, Ty - ty0);
        __syncthreads();
        if (kVec) {  // Ty % 4 == 0, dy 16-byte aligned: every slab row starts 16-byte aligned
            const int tn4 = tn >> 2;
            for (int e = threadIdx.x; e < nc * tn4; e += 256) {
                const int c = e / tn4, q = e - c * tn4;
                const float4 v = *reinterpret_cast<const float4 *>(dy + ((size_t)b * C + c0 + c) * Ty + ty0 + 4 * q);
                *reinterpret_cast<float4 *>(&sdy[c * kErMaxTy + 4 * q]) = v;
            }
        } else {
            for (int e = threadIdx.x; e < nc * tn; e += 256) {
                const int c = e / tn, yy = e - c * tn;
                sdy[c * kErMaxTy + yy] = dy[((size_t)b * C + c0 + c) * Ty + ty0 + yy];
            }
        }
        __syncthreads();
        // 16 lanes per row: a run is summed as 16 strided partial sums + a 4-step xor tree (fixed
        // order, deterministic); a degenerate alignment (one row owning thousands of frames) costs
        // run/16 dependent LDS reads instead of run.
        const int l16 = threadIdx.x & 15;
        for (int e = threadIdx.x >> 4; e < nc * Tx; e += 16) {
            const int c = e / Tx, x = e - c * Tx;
            const int s = rs[x];
            int lo = 0, hi = 0;
            if (s >= 0) {
                const int en = (x == t_x - 1) ? t_y : rs[x + 1];
                lo = max(s, ty0) - ty0;
                hi = min(en, ty0 + tn) - ty0;
            }
            float acc = 0.f;
            for (int yy = lo + l16; yy < hi; yy += 16) acc += sdy[c * kErMaxTy + yy];
            acc += __shfl_xor(acc, 8, 16);
            acc += __shfl_xor(acc, 4, 16);
            acc += __shfl_xor(acc, 2, 16);
            acc += __shfl_xor(acc, 1, 16);
            if (l16 == 0) {
                float *o = dx + ((size_t)b * C + c0 + c) * Tx + x;
                *o = ty0 == 0 ? acc : *o + acc;
            }
        }
    }
}

struct WsLayout {
    size_t lengths, row_start, bits, lat, total;  // lat: the transposed lattice (maximum_path_f32, tr_enabled)
    int K, Txp, nch;
    bool lds_bits;
    int W, KL;  // W > 1: the multi-wave DP (mas_dp_mw_kernel), W waves x KL rows per lane
};

// Whether the DP reads the transposed lattice (column-major loads) for text length Tx: from Tx > 128 (one-wave K >= 4
// and the multi-wave kernels: 8 x 256 x 2048 0.278 -> 0.249 ms, 8 x 512 x 4096 0.930 -> 0.593, 8 x 1024 x 4096 1.90 ->
// 0.93); at K <= 2 rows per lane the row-major loads are not what binds and the transposed copy costs more than
// it saves (32 x 120 x 600, training path: 0.102 vs 0.106 ms; profiles/r04/mas/sweep.jsonl).  MTTS_MAS_TR=0 / 1
// force it off / on; read at every call (a host getenv), so one process can run -- and test -- both layouts.
bool tr_enabled(int Tx) {
    const char *e = getenv("MTTS_MAS_TR");
    if (e && e[0] == '0') return false;
    if (e && e[0] == '1') return true;
    return Tx > 128;
}

// lattice chunks in flight for the one-wave DP on the transposed lattice (MTTS_MAS_TR_RING: 2 / 4 / 8)
int tr_ring() {
    static const int d = [] {
        const char *e = getenv("MTTS_MAS_TR_RING");
        const int v = e ? atoi(e) : 0;
        return (v == 2 || v == 4 || v == 8) ? v : 4;
    }();
    return d;
}

// MTTS_MAS_MW=0: the one-wave DP for every Tx (A/B; Tx <= 2048 then)
bool mw_enabled() {
    static const bool on = [] {
        const char *e = getenv("MTTS_MAS_MW");
        return !(e && e[0] == '0');
    }();
    return on;
}

// shape_override: MTTS_MAS_SHAPE may pick the DP shape -- only where the DP reads the transposed lattice (the
// row-major kernels reject several of the shapes it can name: ADVICE r4)
WsLayout ws_layout(int B, int Tx, int Ty, bool with_lat = false, bool shape_override = true) {
    WsLayout w{};
    w.W = 1;
    w.KL = 1;
    w.K = Tx <= 64 ? 1 : Tx <= 128 ? 2 : Tx <= 256 ? 4 : Tx <= 512 ? 8 : Tx <= 1024 ? 16 : 32;
    w.Txp = kWave * w.K;
    // the multi-wave DP where it measured faster (tools/mas_bench.py, profiles/r04/sweeps/mas_*.jsonl: 8 x 512 x 4096
    // 0.93 vs 0.99 ms) or where the one-wave one cannot go (Tx > 2048); at Tx <= 256 the one-wave kernel is faster
    // (120 x 600: 65 vs 72 us; 256 x 2048: 280 vs 319 us) -- the per-column dependency chain, not the rows per
    // lane, bounds both
    if (Tx > 256 && mw_enabled()) {
        w.W = 8;
        w.KL = Tx <= 512 ? 1 : Tx <= 1024 ? 2 : Tx <= 2048 ? 4 : Tx <= 4096 ? 8 : 16;  // (16: transposed lattice only)
        w.K = w.W * w.KL;
        w.Txp = kWave * w.K;
    }
    // MTTS_MAS_SHAPE="W,KL" (tuning sweeps, transposed-lattice DP only -- every lattice but the core.pyx API's):
    // W waves x KL rows per lane; W = 1 the one-wave kernel (K from Tx).  Ignored unless it covers Tx.
    if (const char *e = shape_override ? getenv("MTTS_MAS_SHAPE") : nullptr) {
        int W = 0, KL = 0;
        if (sscanf(e, "%d,%d", &W, &KL) == 2 && tr_enabled(Tx)) {
            const bool ok1 = W == 1;
            const bool okm = (W == 2 && (KL == 1 || KL == 2)) || (W == 4 && (KL == 1 || KL == 2 || KL == 4)) ||
                             (W == 8 && (KL == 1 || KL == 2 || KL == 4 || KL == 8));
            if (ok1 && Tx <= 2048) {
                w.W = w.KL = 1;
                w.K = Tx <= 64 ? 1 : Tx <= 128 ? 2 : Tx <= 256 ? 4 : Tx <= 512 ? 8 : Tx <= 1024 ? 16 : 32;
                w.Txp = kWave * w.K;
            } else if (okm && kWave * W * KL >= Tx) {
                w.W = W;
                w.KL = KL;
                w.K = W * KL;
                w.Txp = kWave * w.K;
            }
        }
    }
    w.nch = (Ty + 31) / 32;
    w.lds_bits = (size_t)w.Txp * w.nch * 4 <= (size_t)kLdsBitsLimit;
    size_t off = 0;
    w.lengths = off;
    off = mtts::align_up(off + (size_t)B * 2 * 4, 256);
    w.row_start = off;
    off = mtts::align_up(off + (size_t)B * Tx * 4, 256);
    w.bits = off;
    if (!w.lds_bits) off = mtts::align_up(off + (size_t)B * w.nch * w.Txp * 4, 256);
    w.lat = off;
    if (with_lat && tr_enabled(Tx)) off = mtts::align_up(off + (size_t)B * Ty * w.Txp * 4, 256);
    w.total = off;
    return w;
}

// dynamic LDS past 64 KiB needs the kernel attribute (a long Ty's backtrack slot copy: nch x 256 B)
constexpr size_t kMwLdsMax = 160 * 1024 - 256;  // (the kernel's static hand-over flags take the rest)
// global-bits mode: as many backtrack slot buffers (nch x 256 B each, at most 2) as the LDS holds beside `shmem`;
// sets a.bt_bufs and returns the launch's LDS bytes
size_t mw_backtrack_bufs(MasArgs &a, size_t shmem) {
    const size_t slot = (size_t)a.nch * kWave * 4;
    a.bt_bufs = shmem + 2 * slot <= kMwLdsMax ? 2 : shmem + slot <= kMwLdsMax ? 1 : 0;
    return shmem + a.bt_bufs * slot;
}
template <typename K>
bool mw_lds_attr(K kernel, size_t bytes) {
    if (bytes + 256 <= 64 * 1024) return true;  // (+ the static hand-over flags)
    return hipFuncSetAttribute(reinterpret_cast<const void *>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes) == hipSuccess;
}

template <int KL, int W, bool PM>
int launch_dp_mw(MasArgs a, int B, bool vec, bool lds_bits, bool dp_out, size_t shmem, hipStream_t st) {
    dim3 grid(B), block(64 * W);
    if (!lds_bits) shmem = mw_backtrack_bufs(a, shmem);
#define MTTS_MAS_MW_LAUNCH(V, L, DO)                                                                  \
    do {                                                                                              \
        if (!mw_lds_attr(mas_dp_mw_kernel<KL, W, PM, V, L, DO && PM>, shmem))                         \
            return mtts::fail(MTTS_ERR_HIP, "maximum_path: LDS attribute");                           \
        hipLaunchKernelGGL((mas_dp_mw_kernel<KL, W, PM, V, L, DO && PM>), grid, block, shmem, st, a); \
    } while (0)
    if (vec) {
        if (lds_bits) {
            if (dp_out) MTTS_MAS_MW_LAUNCH(true, true, true); else MTTS_MAS_MW_LAUNCH(true, true, false);
        } else {
            if (dp_out) MTTS_MAS_MW_LAUNCH(true, false, true); else MTTS_MAS_MW_LAUNCH(true, false, false);
        }
    } else {
        if (lds_bits) {
            if (dp_out) MTTS_MAS_MW_LAUNCH(false, true, true); else MTTS_MAS_MW_LAUNCH(false, true, false);
        } else {
            if (dp_out) MTTS_MAS_MW_LAUNCH(false, false, true); else MTTS_MAS_MW_LAUNCH(false, false, false);
        }
    }
#undef MTTS_MAS_MW_LAUNCH
    return mtts::check_launch("mas_dp_mw_kernel");
}

template <int KL, int W>
int launch_dp_mw_pm(const MasArgs &a, int B, bool vec, bool lds_bits, bool dp_out, size_t shmem, hipStream_t st) {
    if (!a.premasked) {
        if (dp_out) return mtts::fail(MTTS_ERR_INVALID_ARG, "maximum_path: dp_out needs a premasked lattice");
        return launch_dp_mw<KL, W, false>(a, B, vec, lds_bits, false, shmem, st);
    }
    return launch_dp_mw<KL, W, true>(a, B, vec, lds_bits, dp_out, shmem, st);
}

template <int K, int C, int D, bool PM>
int launch_dp_k(const MasArgs &a, int B, bool vec, bool lds_bits, bool dp_out, size_t shmem, hipStream_t st) {
    dim3 grid(B), block(kWave);
#define MTTS_MAS_LAUNCH(V, L, DO) \
    hipLaunchKernelGGL((mas_dp_kernel<K, C, D, PM, V, L, DO && PM>), grid, block, shmem, st, a)
    if (vec) {
        if (lds_bits) {
            if (dp_out) MTTS_MAS_LAUNCH(true, true, true); else MTTS_MAS_LAUNCH(true, true, false);
        } else {
            if (dp_out) MTTS_MAS_LAUNCH(true, false, true); else MTTS_MAS_LAUNCH(true, false, false);
        }
    } else {
        if (lds_bits) {
            if (dp_out) MTTS_MAS_LAUNCH(false, true, true); else MTTS_MAS_LAUNCH(false, true, false);
        } else {
            if (dp_out) MTTS_MAS_LAUNCH(false, false, true); else MTTS_MAS_LAUNCH(false, false, false);
        }
    }
#undef MTTS_MAS_LAUNCH
    return mtts::check_launch("mas_dp_kernel");
}

// Chunk shape and ring depth per rows-per-lane K: K*C = 32 cells per lane per chunk; the premasked
// lattice (the fused training path and core.pyx's API) carries no mask registers, so it affords a
// deeper ring.  MTTS_MAS_RING overrides the premasked depth (tuning).
int ring_depth() {
    static const int d = [] {
        const char *e = getenv("MTTS_MAS_RING");
        const int v = e ? atoi(e) : 0;
        return (v == 2 || v == 3 || v == 4) ? v : 0;
    }();
    return d;
}

template <int K, int C>
int launch_dp_kc(const MasArgs &a, int B, bool vec, bool lds_bits, bool dp_out, size_t shmem, hipStream_t st) {
    if (!a.premasked) {
        if (dp_out) return mtts::fail(MTTS_ERR_INVALID_ARG, "maximum_path: dp_out needs a premasked lattice");
        return launch_dp_k<K, C, 2, false>(a, B, vec, lds_bits, false, shmem, st);
    }
    const int d = ring_depth() ? ring_depth() : kDefaultRing;
    if (d == 2) return launch_dp_k<K, C, 2, true>(a, B, vec, lds_bits, dp_out, shmem, st);
    if (d == 3) return launch_dp_k<K, C, 3, true>(a, B, vec, lds_bits, dp_out, shmem, st);
    return launch_dp_k<K, C, 4, true>(a, B, vec, lds_bits, dp_out, shmem, st);
}

template <int KL, int W>
int launch_dp_mw_tr(MasArgs a, int B, bool lds_bits, size_t shmem, hipStream_t st) {
    if (!lds_bits) shmem = mw_backtrack_bufs(a, shmem);
    if constexpr (KL <= 8) {  // (KL = 16: Txp = 8192 rows never fit the LDS-bits budget)
        if (lds_bits) {
            if (!mw_lds_attr(mas_dp_mw_kernel<KL, W, true, false, true, false, true>, shmem))
                return mtts::fail(MTTS_ERR_HIP, "maximum_path: LDS attribute");
            hipLaunchKernelGGL((mas_dp_mw_kernel<KL, W, true, false, true, false, true>), dim3(B), dim3(64 * W), shmem, st, a);
            return mtts::check_launch("mas_dp_mw_kernel");
        }
    }
    {
        if (!mw_lds_attr(mas_dp_mw_kernel<KL, W, true, false, false, false, true>, shmem))
            return mtts::fail(MTTS_ERR_HIP, "maximum_path: LDS attribute");
        hipLaunchKernelGGL((mas_dp_mw_kernel<KL, W, true, false, false, false, true>), dim3(B), dim3(64 * W), shmem, st, a);
    }
    return mtts::check_launch("mas_dp_mw_kernel");
}

template <int K, int C, int D>
int launch_dp_k_tr(const MasArgs &a, int B, bool lds_bits, size_t shmem, hipStream_t st) {
    if (lds_bits)
        hipLaunchKernelGGL((mas_dp_kernel<K, C, D, true, false, true, false, true>), dim3(B), dim3(kWave), shmem, st, a);
    else
        hipLaunchKernelGGL((mas_dp_kernel<K, C, D, true, false, false, false, true>), dim3(B), dim3(kWave), shmem, st, a);
    return mtts::check_launch("mas_dp_kernel");
}

template <int K, int C>
int launch_dp_kc_tr(const MasArgs &a, int B, bool lds_bits, size_t shmem, hipStream_t st) {
    const int d = tr_ring();
    if (d == 2) return launch_dp_k_tr<K, C, 2>(a, B, lds_bits, shmem, st);
    if (d == 8) return launch_dp_k_tr<K, C, 8>(a, B, lds_bits, shmem, st);
    return launch_dp_k_tr<K, C, 4>(a, B, lds_bits, shmem, st);
}

// The DP on the transposed premasked lattice (a.tr_ld > 0): same kernels, column-major loads
int launch_dp_tr(const MasArgs &a, int B, const WsLayout &w, hipStream_t st) {
    if (w.W > 1) {
        const size_t shmem = (size_t)w.Txp * 4 + (size_t)kEdgeRing * w.W * 32 * 4 + (w.lds_bits ? (size_t)w.Txp * w.nch * 4 : 0);
        if (w.W == 2) return w.KL == 2 ? launch_dp_mw_tr<2, 2>(a, B, w.lds_bits, shmem, st)
                                       : launch_dp_mw_tr<1, 2>(a, B, w.lds_bits, shmem, st);
        if (w.W == 4) return w.KL == 4   ? launch_dp_mw_tr<4, 4>(a, B, w.lds_bits, shmem, st)
                             : w.KL == 2 ? launch_dp_mw_tr<2, 4>(a, B, w.lds_bits, shmem, st)
                                         : launch_dp_mw_tr<1, 4>(a, B, w.lds_bits, shmem, st);
        switch (w.KL) {
            case 1: return launch_dp_mw_tr<1, 8>(a, B, w.lds_bits, shmem, st);
            case 2: return launch_dp_mw_tr<2, 8>(a, B, w.lds_bits, shmem, st);
            case 4: return launch_dp_mw_tr<4, 8>(a, B, w.lds_bits, shmem, st);
            case 8: return launch_dp_mw_tr<8, 8>(a, B, w.lds_bits, shmem, st);
            default: return launch_dp_mw_tr<16, 8>(a, B, false, shmem, st);  // Tx <= 8192 (global bits)
        }
    }
    const size_t shmem = (size_t)w.Txp * 4 + (w.lds_bits ? (size_t)w.Txp * w.nch * 4 : 0);
    switch (w.K) {
        case 1: return launch_dp_kc_tr<1, 32>(a, B, w.lds_bits, shmem, st);
        case 2: return launch_dp_kc_tr<2, 16>(a, B, w.lds_bits, shmem, st);
        case 4: return launch_dp_kc_tr<4, 8>(a, B, w.lds_bits, shmem, st);
        case 8: return launch_dp_kc_tr<8, 4>(a, B, w.lds_bits, shmem, st);
        case 16: return launch_dp_kc_tr<16, 2>(a, B, w.lds_bits, shmem, st);
        default: return launch_dp_kc_tr<32, 1>(a, B, w.lds_bits, shmem, st);
    }
}

int launch_dp(MasArgs a, int B, const WsLayout &w, bool vec, bool dp_out, hipStream_t st) {
    if (a.tr_ld > 0) return dp_out ? mtts::fail(MTTS_ERR_INVALID_ARG, "maximum_path: dp_out needs the row-major lattice")
                                   : launch_dp_tr(a, B, w, st);
    if (w.W > 1) {
        const size_t shmem = (size_t)w.Txp * 4 + (size_t)kEdgeRing * w.W * 32 * 4 + (w.lds_bits ? (size_t)w.Txp * w.nch * 4 : 0);
        if (w.W < 8 && w.KL != 1) return mtts::fail(MTTS_ERR_UNSUPPORTED, "maximum_path: DP shape needs the transposed lattice");
        if (w.KL > 8)
            return mtts::fail(MTTS_ERR_SHAPE, "maximum_path: Tx > 4096 needs the transposed lattice (compute_batch_alignments / "
                                              "dp_out and MTTS_MAS_TR=0 keep the row-major lattice: Tx <= 4096)");
        if (w.W == 2) return launch_dp_mw_pm<1, 2>(a, B, vec, w.lds_bits, dp_out, shmem, st);
        if (w.W == 4) return launch_dp_mw_pm<1, 4>(a, B, vec, w.lds_bits, dp_out, shmem, st);
        switch (w.KL) {
            case 1: return launch_dp_mw_pm<1, 8>(a, B, vec, w.lds_bits, dp_out, shmem, st);
            case 2: return launch_dp_mw_pm<2, 8>(a, B, vec, w.lds_bits, dp_out, shmem, st);
            case 4: return launch_dp_mw_pm<4, 8>(a, B, vec, w.lds_bits, dp_out, shmem, st);
            default: return launch_dp_mw_pm<8, 8>(a, B, vec, w.lds_bits, dp_out, shmem, st);  // Tx <= 4096
        }
    }
    size_t shmem = (size_t)w.Txp * 4 + (w.lds_bits ? (size_t)w.Txp * w.nch * 4 : 0);
    switch (w.K) {
        case 1: return launch_dp_kc<1, 32>(a, B, vec, w.lds_bits, dp_out, shmem, st);
        case 2: return launch_dp_kc<2, 16>(a, B, vec, w.lds_bits, dp_out, shmem, st);
        case 4: return launch_dp_kc<4, 8>(a, B, vec, w.lds_bits, dp_out, shmem, st);
        case 8: return launch_dp_kc<8, 4>(a, B, vec, w.lds_bits, dp_out, shmem, st);
        case 16: return launch_dp_kc<16, 2>(a, B, vec, w.lds_bits, dp_out, shmem, st);
        default: return launch_dp_kc<32, 1>(a, B, vec, w.lds_bits, dp_out, shmem, st);  // Tx <= 2048
    }
}

int check_shape(int B, int Tx, int Ty) {
    if (B < 0 || Tx < 1 || Ty < 1) return mtts::fail(MTTS_ERR_INVALID_ARG, "maximum_path: bad shape");
    if (Tx > MTTS_MAS_MAX_TX || (Tx > 2048 && !mw_enabled()))
        return mtts::fail(MTTS_ERR_SHAPE, "maximum_path: Tx > MTTS_MAS_MAX_TX (8192) is not supported");
    if ((int64_t)Tx * Ty * 4 >= (int64_t)1 << 31)
        return mtts::fail(MTTS_ERR_SHAPE, "maximum_path: one utterance's lattice exceeds 2 GiB");
    return MTTS_OK;
}

}  // namespace

extern "C" size_t mtts_maximum_path_workspace_size(int32_t B, int32_t Tx, int32_t Ty) {
    if (B < 0 || Tx < 1 || Ty < 1) return 0;
    // covers maximum_path (transposed lattice where tr_enabled) and compute_batch_alignments (row-major)
    return std::max(ws_layout(B, Tx, Ty, true).total, ws_layout(B, Tx, Ty, true, false).total);
}

extern "C" int mtts_maximum_path_f32(const float *value, const float *mask, float *path, int32_t B,
                                     int32_t Tx, int32_t Ty, int32_t flags, int32_t *lengths_out,
                                     int32_t *row_start_out, void *workspace, size_t workspace_bytes,
                                     void *hip_stream) {
    int rc = check_shape(B, Tx, Ty);
    if (rc) return rc;
    MTTS_CHECK_ARG((flags & ~(MTTS_MAS_VALUE_PREMASKED | MTTS_MAS_NO_DENSE_PATH)) == 0,
                   "maximum_path: unknown flag bits");
    if (B == 0) return MTTS_OK;
    MTTS_CHECK_ARG(value && mask, "maximum_path: value and mask are required");
    MTTS_CHECK_ARG(path || (flags & MTTS_MAS_NO_DENSE_PATH), "maximum_path: path is null");
    const WsLayout w = ws_layout(B, Tx, Ty, true);
    if (!workspace || workspace_bytes < w.total)
        return mtts::fail(MTTS_ERR_WORKSPACE, "maximum_path: workspace too small");
    char *ws = static_cast<char *>(workspace);
    hipStream_t st = static_cast<hipStream_t>(hip_stream);

    MasArgs a{};
    a.value = value;
    a.mask = mask;
    if (tr_enabled(Tx)) {  // premask + transpose once (coalesced), then the DP's column-major loads
        float *lat = reinterpret_cast<float *>(ws + w.lat);
        const bool pm = flags & MTTS_MAS_VALUE_PREMASKED;
        hipLaunchKernelGGL(mas_transpose_kernel, dim3((Ty + 63) / 64, w.Txp / 64, B), dim3(256), 0, st, value,
                           pm ? nullptr : mask, Tx, Ty, w.Txp, lat);
        rc = mtts::check_launch("mas_transpose_kernel");
        if (rc) return rc;
        a.value = lat;
        a.tr_ld = w.Txp;
    }
    a.lengths = lengths_out ? lengths_out : reinterpret_cast<int32_t *>(ws + w.lengths);
    a.row_start = row_start_out ? row_start_out : reinterpret_cast<int32_t *>(ws + w.row_start);
    a.bits = reinterpret_cast<uint32_t *>(ws + w.bits);
    a.Tx = Tx;
    a.Ty = Ty;
    a.Txp = w.Txp;
    a.nch = w.nch;
    a.premasked = (flags & MTTS_MAS_VALUE_PREMASKED) || a.tr_ld ? 1 : 0;
    a.neg = -1e9f;
    const bool vec = (Ty % 4 == 0) && ((uintptr_t)value % 16 == 0) &&
                     (a.premasked || (uintptr_t)mask % 16 == 0);
    rc = launch_dp(a, B, w, vec, false, st);
    if (rc || (flags & MTTS_MAS_NO_DENSE_PATH)) return rc;

    dim3 grid((Ty + 1023) / 1024, Tx, B);
    const int vec4 = (Ty % 4 == 0) && ((uintptr_t)path % 16 == 0);
    hipLaunchKernelGGL((mas_expand_kernel<float, false>), grid, dim3(256), 0, st, a.row_start,
                       a.lengths, path, Tx, Ty, vec4);
    return mtts::check_launch("mas_expand_kernel");
}

extern "C" size_t mtts_prior_maximum_path_workspace_size(int32_t B, int32_t Tx, int32_t Ty) {
    if (B < 0 || Tx < 1 || Ty < 1) return 0;
    size_t n = 0;
    for (const bool tr : {true, false}) {  // the layout of either lattice (the call may pass lattice_out or not)
        const WsLayout w = ws_layout(B, Tx, Ty, false, tr);  // lattice: row-major [B,Tx,Ty] or transposed [B,Ty,Txp]
        n = std::max(n, mtts::align_up(w.total, 256) + mtts::align_up((size_t)B * 2 * 4, 256) +
                            (size_t)B * Ty * (Tx > w.Txp ? Tx : w.Txp) * 4);
    }
    return n;
}

extern "C" int mtts_prior_maximum_path(const float *mu_x, const float *y, const int64_t *x_lengths,
                                       const int64_t *y_lengths, int32_t B, int32_t C, int32_t Tx, int32_t Ty,
                                       float *path, int32_t *lengths_out, int32_t *row_start_out, float *dur_out,
                                       int32_t *col_row_out, float *lattice_out, void *workspace,
                                       size_t workspace_bytes, void *hip_stream) {
    int rc = check_shape(B, Tx, Ty);
    if (rc) return rc;
    if (B == 0) return MTTS_OK;
    MTTS_CHECK_ARG(mu_x && y && x_lengths && y_lengths && C >= 1, "prior_maximum_path: null input or C < 1");
    MTTS_CHECK_ARG(B <= 65535, "prior_maximum_path: B > 65535");
    const WsLayout w = ws_layout(B, Tx, Ty, false, !lattice_out);  // a caller lattice_out is row-major
    if (!workspace || workspace_bytes < mtts_prior_maximum_path_workspace_size(B, Tx, Ty))
        return mtts::fail(MTTS_ERR_WORKSPACE, "prior_maximum_path: workspace too small");
    char *ws = static_cast<char *>(workspace);
    const size_t o_txy = mtts::align_up(w.total, 256), o_lat = o_txy + mtts::align_up((size_t)B * 2 * 4, 256);
    int32_t *txy = reinterpret_cast<int32_t *>(ws + o_txy);
    float *lat = lattice_out ? lattice_out : reinterpret_cast<float *>(ws + o_lat);
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    // the lattice the caller does not see is written transposed for the DP's column-major loads
    const bool tr = !lattice_out && tr_enabled(Tx);

    const float cst = (float)(-0.5 * std::log(2.0 * M_PI) * C);  // the Python scalar, rounded as torch does
    dim3 lg((Ty + kLpT - 1) / kLpT, ((tr ? w.Txp : Tx) + kLpT - 1) / kLpT, B);
    if (tr)
        hipLaunchKernelGGL(log_prior_kernel<true>, lg, dim3(256), 0, st, mu_x, y, x_lengths, y_lengths, C, Tx, Ty, cst,
                           lat, txy, w.Txp);
    else
        hipLaunchKernelGGL(log_prior_kernel<false>, lg, dim3(256), 0, st, mu_x, y, x_lengths, y_lengths, C, Tx, Ty, cst,
                           lat, txy, 0);
    rc = mtts::check_launch("log_prior_kernel");
    if (rc) return rc;

    MasArgs a{};
    a.value = lat;
    a.t_xs = txy;
    a.t_ys = txy + B;
    a.lengths = lengths_out ? lengths_out : reinterpret_cast<int32_t *>(ws + w.lengths);
    a.row_start = row_start_out ? row_start_out : reinterpret_cast<int32_t *>(ws + w.row_start);
    a.bits = reinterpret_cast<uint32_t *>(ws + w.bits);
    a.Tx = Tx;
    a.Ty = Ty;
    a.Txp = w.Txp;
    a.nch = w.nch;
    a.premasked = 1;
    a.neg = -1e9f;
    a.tr_ld = tr ? w.Txp : 0;
    const bool vec = (Ty % 4 == 0) && ((uintptr_t)lat % 16 == 0);
    rc = launch_dp(a, B, w, vec, false, st);
    if (rc) return rc;
    if (path) {
        dim3 grid((Ty + 1023) / 1024, Tx, B);
        const int vec4 = (Ty % 4 == 0) && ((uintptr_t)path % 16 == 0);
        hipLaunchKernelGGL((mas_expand_kernel<float, false>), grid, dim3(256), 0, st, a.row_start, a.lengths, path, Tx,
                           Ty, vec4);
        rc = mtts::check_launch("mas_expand_kernel");
        if (rc) return rc;
    }
    if (dur_out || col_row_out) {
        hipLaunchKernelGGL(mas_runs_kernel, dim3(B), dim3(256), 0, st, a.row_start, a.lengths, Tx, Ty, dur_out,
                           col_row_out);
        rc = mtts::check_launch("mas_runs_kernel");
    }
    return rc;
}

extern "C" int mtts_expand_rows_fwd(const float *src, const int32_t *col_row, int32_t B, int32_t C, int32_t Tx,
                                    int32_t Ty, float *dst, void *hip_stream) {
    MTTS_CHECK_ARG(src && col_row && dst && B >= 0 && C >= 0 && Tx >= 1 && Ty >= 0 && B <= 65535,
                   "expand_rows_fwd: bad args");
    if ((size_t)B * C * Ty == 0) return MTTS_OK;
    dim3 grid((unsigned)(((size_t)C * Ty + 255) / 256), B);
    hipLaunchKernelGGL(expand_rows_fwd_kernel, grid, dim3(256), 0, static_cast<hipStream_t>(hip_stream), src, col_row,
                       C, Tx, Ty, dst);
    return mtts::check_launch("expand_rows_fwd_kernel");
}

extern "C" int mtts_expand_rows_bwd(const float *dy, const int32_t *row_start, const int32_t *lengths, int32_t B,
                                    int32_t C, int32_t Tx, int32_t Ty, float *dx, void *hip_stream) {
    MTTS_CHECK_ARG(dy && row_start && lengths && dx && B >= 0 && C >= 0 && Tx >= 1 && Ty >= 1 && B <= 65535,
                   "expand_rows_bwd: bad args");
    if ((size_t)B * C * Tx == 0) return MTTS_OK;
    dim3 grid((unsigned)((C + kErC - 1) / kErC), B);
    const bool vec = (Ty % 4 == 0) && ((uintptr_t)dy % 16 == 0);
    if (vec)
        hipLaunchKernelGGL(expand_rows_bwd_kernel<true>, grid, dim3(256), 0, static_cast<hipStream_t>(hip_stream), dy,
                           row_start, lengths, C, Tx, Ty, dx);
    else
        hipLaunchKernelGGL(expand_rows_bwd_kernel<false>, grid, dim3(256), 0, static_cast<hipStream_t>(hip_stream), dy,
                           row_start, lengths, C, Tx, Ty, dx);
    return mtts::check_launch("expand_rows_bwd_kernel");
}

extern "C" int mtts_compute_batch_alignments(int32_t *paths, float *values, const int32_t *t_xs,
                                             const int32_t *t_ys, int32_t B, int32_t Tx, int32_t Ty,
                                             float max_neg_val, void *workspace,
                                             size_t workspace_bytes, void *hip_stream) {
    int rc = check_shape(B, Tx, Ty);
    if (rc) return rc;
    if (B == 0) return MTTS_OK;
    MTTS_CHECK_ARG(paths && values && t_xs && t_ys, "compute_batch_alignments: null pointer");
    const WsLayout w = ws_layout(B, Tx, Ty, false, false);  // row-major lattice (the in-place core.pyx API)
    if (!workspace || workspace_bytes < w.total)
        return mtts::fail(MTTS_ERR_WORKSPACE, "compute_batch_alignments: workspace too small");
    char *ws = static_cast<char *>(workspace);
    hipStream_t st = static_cast<hipStream_t>(hip_stream);

    MasArgs a{};
    a.value = values;
    a.mask = nullptr;
    a.t_xs = t_xs;
    a.t_ys = t_ys;
    a.lengths = reinterpret_cast<int32_t *>(ws + w.lengths);
    a.row_start = reinterpret_cast<int32_t *>(ws + w.row_start);
    a.bits = reinterpret_cast<uint32_t *>(ws + w.bits);
    a.dp_out = values;  // in place, exactly like the Cython (core.pyx:83-85)
    a.Tx = Tx;
    a.Ty = Ty;
    a.Txp = w.Txp;
    a.nch = w.nch;
    a.premasked = 1;
    a.neg = max_neg_val;
    const bool vec = (Ty % 4 == 0) && ((uintptr_t)values % 16 == 0);
    rc = launch_dp(a, B, w, vec, true, st);
    if (rc) return rc;
    dim3 grid((Ty + 1023) / 1024, Tx, B);
    hipLaunchKernelGGL((mas_expand_kernel<int32_t, true>), grid, dim3(256), 0, st, a.row_start,
                       a.lengths, paths, Tx, Ty, 0);
    return mtts::check_launch("mas_expand_kernel");
}
