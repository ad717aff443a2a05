// Batched weight packing: every GEMM operand layout the decoder step needs, in a few launches.
//
// The implicit-GEMM kernels read weights as [rows][ld] with K ordered tap-major / channel-minor
// (k' = j*C + c) in the operand precision.  torch keeps Conv1d weights [Cout][Cin][k], ConvTranspose1d
// [Cin][Cout][k] and Linear [N][K] in fp32; the forward, the dgrad (transposed) and the stride-2
// phase GEMMs each need their own gather of them.  One job = one affine gather
//     dst[r*ld + j*C + c] = src[r*sr + c*sc + (j0 + j*js)*sj],   zero for k' in [C*ntaps, Kp),
// and a launch runs up to kJobsPerLaunch jobs (blockIdx.y = job), each thread producing 8
// consecutive k' (one 16-byte bf16 store, or two float4).  bf16 jobs with lo_off > 0 also write the
// rounding residual bf16(w - bf16(w)) as a second plane (MTTS_GEMM_F_W_SPLIT operands), and with
// MTTS_PACK_THREE_PLANES a third, bf16(w - hi - mid): hi + mid + lo == w exactly (MTTS_GEMM_F_SPLIT3).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

constexpr int kJobsPerLaunch = 32;
constexpr int kThreads = 256;

struct JobBatch {
    mtts_pack_job job[kJobsPerLaunch];
};

template <bool BF16>
__device__ __forceinline__ void pack_tiles(const mtts_pack_job &j, float (*tile)[65]);
__host__ __device__ inline bool tiled_job(const mtts_pack_job &j);

template <bool BF16>
__global__ __launch_bounds__(kThreads) void pack_kernel(JobBatch jb) {
    const mtts_pack_job &j = jb.job[blockIdx.y];
    if (tiled_job(j)) {  // job-uniform branch
        __shared__ float tile[32][65];
        pack_tiles<BF16>(j, tile);
        return;
    }
    const int groups = j.Kp / 8;
    const long total = (long)j.rows * groups;
    const int K = j.C * j.ntaps;
    for (long gi = (long)blockIdx.x * kThreads + threadIdx.x; gi < total; gi += (long)gridDim.x * kThreads) {
        const int r = (int)(gi / groups);
        const int k0 = (int)(gi - (long)r * groups) * 8;
        int tap = k0 / j.C, c = k0 - tap * j.C;
        float e[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            e[i] = k0 + i < K ? j.src[(int64_t)r * j.sr + (int64_t)c * j.sc + (int64_t)(j.j0 + tap * j.js) * j.sj]
                              : 0.f;
            if (++c == j.C) {
                c = 0;
                ++tap;
            }
        }
        if constexpr (BF16) {
            const bool three = (j.lo_off & MTTS_PACK_THREE_PLANES) != 0;
            const int64_t off = j.lo_off & ~MTTS_PACK_THREE_PLANES;
            uint32_t w[4], l[4], l2[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const __bf16 h0 = (__bf16)e[2 * i], h1 = (__bf16)e[2 * i + 1];
                w[i] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
                // split plane: the rounding residual, exact in fp32 (e - hi has <= 16 significant bits)
                const float r0 = e[2 * i] - (float)h0, r1 = e[2 * i + 1] - (float)h1;
                const __bf16 l0 = (__bf16)r0, l1 = (__bf16)r1;
                l[i] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
                // third plane (bf16x6): what the mid plane leaves, <= 8 significant bits -- exact in bf16
                const __bf16 m0 = (__bf16)(r0 - (float)l0), m1 = (__bf16)(r1 - (float)l1);
                l2[i] = (uint32_t)__builtin_bit_cast(uint16_t, m0) | ((uint32_t)__builtin_bit_cast(uint16_t, m1) << 16);
            }
            uint16_t *d = static_cast<uint16_t *>(j.dst) + (size_t)r * j.ld + k0;
            *reinterpret_cast<uint4 *>(d) = make_uint4(w[0], w[1], w[2], w[3]);
            if (off > 0) *reinterpret_cast<uint4 *>(d + off) = make_uint4(l[0], l[1], l[2], l[3]);
            if (three) *reinterpret_cast<uint4 *>(d + 2 * off) = make_uint4(l2[0], l2[1], l2[2], l2[3]);
        } else {
            float4 *d = reinterpret_cast<float4 *>(static_cast<float *>(j.dst) + (size_t)r * j.ld + k0);
            d[0] = make_float4(e[0], e[1], e[2], e[3]);
            d[1] = make_float4(e[4], e[5], e[6], e[7]);
        }
    }
}

// Transposing jobs (sc > sr: a dgrad layout gathers a weight COLUMN per destination row, e.g. the linear
// dgrad's sc = K) read one 4-byte element per 8 destination elements from lines they barely use.  Tiled
// here: 32 destination rows x 64 c of one tap are read with the destination ROW fastest across threads
// (src stride sr: 1 or k), transposed through LDS, and written as 16-byte row segments.  C % 8 == 0
// (every 8-element group lies inside one tap), Kp == C * ntaps (no padding to zero), 16-byte aligned dst.
constexpr int kTR = 32, kTC = 64;

template <bool BF16>
__device__ __forceinline__ void pack_tiles(const mtts_pack_job &j, float (*tile)[kTC + 1]) {
    const int rt = (j.rows + kTR - 1) / kTR, ct = (j.C + kTC - 1) / kTC;
    const long ntile = (long)rt * ct * j.ntaps;
    const int tid = threadIdx.x;
    for (long t = blockIdx.x; t < ntile; t += gridDim.x) {
        const int tap = (int)(t / ((long)rt * ct)), rem = (int)(t - (long)tap * rt * ct);
        const int r0 = (rem / ct) * kTR, c0 = (rem % ct) * kTC;
        const float *src = j.src + (int64_t)(j.j0 + tap * j.js) * j.sj;
        __syncthreads();  // the previous tile's LDS reads are done
#pragma unroll
        for (int i = 0; i < kTR * kTC / kThreads; ++i) {  // load: destination row fastest (src stride sr)
            const int e = tid + kThreads * i, rr = e % kTR, cc = e / kTR;
            const int r = r0 + rr, c = c0 + cc;
            tile[rr][cc] = (r < j.rows && c < j.C) ? src[(int64_t)r * j.sr + (int64_t)c * j.sc] : 0.f;
        }
        __syncthreads();
        const int rr = tid / (kTC / 8), g = tid % (kTC / 8);  // 32 rows x 8 groups of 8 = 256 threads
        const int r = r0 + rr, c = c0 + 8 * g;
        if (r >= j.rows || c >= j.C) continue;
        float e[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) e[q] = tile[rr][8 * g + q];
        const size_t off = (size_t)r * j.ld + (size_t)tap * j.C + c;
        if constexpr (BF16) {
            uint32_t w[4], l[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const __bf16 h0 = (__bf16)e[2 * q], h1 = (__bf16)e[2 * q + 1];
                w[q] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
                const __bf16 l0 = (__bf16)(e[2 * q] - (float)h0), l1 = (__bf16)(e[2 * q + 1] - (float)h1);
                l[q] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
            }
            uint16_t *d = static_cast<uint16_t *>(j.dst) + off;
            *reinterpret_cast<uint4 *>(d) = make_uint4(w[0], w[1], w[2], w[3]);
            if (j.lo_off > 0) *reinterpret_cast<uint4 *>(d + j.lo_off) = make_uint4(l[0], l[1], l[2], l[3]);
        } else {
            float4 *d = reinterpret_cast<float4 *>(static_cast<float *>(j.dst) + off);
            d[0] = make_float4(e[0], e[1], e[2], e[3]);
            d[1] = make_float4(e[4], e[5], e[6], e[7]);
        }
    }
}

__host__ __device__ inline bool tiled_job(const mtts_pack_job &j) {
    return j.sc > j.sr && j.C % 8 == 0 && j.Kp == j.C * j.ntaps && ((uintptr_t)j.dst & 15) == 0;
}

}  // namespace

extern "C" int mtts_pack_weights(const mtts_pack_job *jobs, int32_t njobs, int32_t precision, void *hip_stream) {
    MTTS_CHECK_ARG(njobs >= 0 && (jobs || njobs == 0), "pack_weights: bad job list");
    MTTS_CHECK_ARG(precision == MTTS_PREC_FP32 || precision == MTTS_PREC_BF16, "pack_weights: bad precision");
    long max_groups = 0;
    for (int i = 0; i < njobs; ++i) {
        const mtts_pack_job &j = jobs[i];
        MTTS_CHECK_ARG(j.src && j.dst, "pack_weights: null pointer");
        MTTS_CHECK_ARG(j.rows >= 0 && j.C >= 1 && j.ntaps >= 1 && j.Kp % 8 == 0 && j.Kp >= j.C * j.ntaps &&
                           j.ld % 8 == 0 && j.ld >= j.Kp,
                       "pack_weights: bad job shape (Kp, ld multiples of 8, Kp >= C*ntaps, ld >= Kp)");
        MTTS_CHECK_ARG((reinterpret_cast<uintptr_t>(j.dst) & 15) == 0, "pack_weights: dst must be 16-byte aligned");
        MTTS_CHECK_ARG(j.lo_off >= 0 && j.lo_off % 8 == 0 && (j.lo_off == 0 || precision == MTTS_PREC_BF16),
                       "pack_weights: lo_off (the split plane) needs bf16 and a multiple of 8");
        MTTS_CHECK_ARG(!(j.lo_off & MTTS_PACK_THREE_PLANES) ||
                           ((j.lo_off & ~MTTS_PACK_THREE_PLANES) > 0 && !tiled_job(j)),
                       "pack_weights: three planes need a plane offset and a non-transposing (forward) layout");
        const long g = (long)j.rows * (j.Kp / 8);
        max_groups = g > max_groups ? g : max_groups;
    }
    if (njobs == 0 || max_groups == 0) return MTTS_OK;
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    for (int base = 0; base < njobs; base += kJobsPerLaunch) {
        const int n = njobs - base < kJobsPerLaunch ? njobs - base : kJobsPerLaunch;
        // blocks per job: one per 256 groups of the launch's largest job, up to ~4096 workgroups per launch (the
        // old cap of 256 per job left a launch of small jobs at <1 workgroup per CU and a large job grid-striding)
        long mg = 0;
        for (int i = 0; i < n; ++i) {
            const long g = (long)jobs[base + i].rows * (jobs[base + i].Kp / 8);
            mg = g > mg ? g : mg;
        }
        const long cap = 4096 / n > 256 ? 4096 / n : 256;
        const int gx = (int)((mg + kThreads - 1) / kThreads < cap ? (mg + kThreads - 1) / kThreads : cap);
        JobBatch jb;
        for (int i = 0; i < n; ++i) jb.job[i] = jobs[base + i];
        if (precision == MTTS_PREC_BF16)
            hipLaunchKernelGGL(pack_kernel<true>, dim3(gx, n), dim3(kThreads), 0, st, jb);
        else
            hipLaunchKernelGGL(pack_kernel<false>, dim3(gx, n), dim3(kThreads), 0, st, jb);
        if (int rc = mtts::check_launch("pack_kernel")) return rc;
    }
    return MTTS_OK;
}
