// L2 -> LDS fill-rate probe (round 5): how many bytes per CU per second LDS-DMA (buffer_load ... lds, 16 B
// per lane) moves for the operand patterns of the conv GEMMs, no MFMA.  Each workgroup streams `steps`
// K steps of STEP bytes through a ring of S LDS buffers (counted vmcnt, raw barrier), as the GEMM main
// loops do.  Patterns (the source address of lane l of DMA instruction i in step k):
//   0 W image shared: rows of 128 B (8 lanes per row), row stride RS bytes; all workgroups read the SAME
//     rows, K advancing 128 B per step (the packed-weight stream every M tile re-reads)
//   1 the same with each workgroup starting at a different K step (rotated)
//   2 shared, contiguous 1 KiB per instruction
//   3 each workgroup its own contiguous region (HBM stream)
//   4 A image: 64-row tiles of 128-B rows, row stride 512 B, workgroup w reads rows 64w.. (tap-free A)
// hipcc --offload-arch=gfx950 -O3 -o tools/bin/fill_probe tools/r5/fill_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 make_rsrc(const void *base, uint32_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)base;
    u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    r.z = __builtin_amdgcn_readfirstlane(bytes);
    r.w = 0x00020000u;
    return r;
}

__device__ __forceinline__ void bload16(uint32_t voff, u32x4 rsrc, uint32_t soff, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
        : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// STEP bytes per K step, S stages, NT threads; INS = DMA instructions per thread per step
template <int STEP, int S, int NT>
__global__ __launch_bounds__(NT) void fill_kernel(const char *src, uint32_t src_bytes, int mode, int steps, int rs,
                                                  float *sink) {
    constexpr int INS = STEP / (NT * 16);
    static_assert(INS * NT * 16 == STEP, "step");
    __shared__ __attribute__((aligned(1024))) char lds[S * STEP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int NW = NT / 64;
    const u32x4 rsrc = make_rsrc(src, src_bytes);
    const uint32_t lbase = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)lds);
    uint32_t voff[INS];
    int kstep0 = 0;
    const int nk = rs / 128;  // K steps per W row
    if (mode == 1) kstep0 = blockIdx.x % nk;
#pragma unroll
    for (int i = 0; i < INS; ++i) {
        const int q = i * NW + wave;  // instruction index within the step
        if (mode == 0 || mode == 1) {
            const int row = q * 8 + lane / 8;  // 8 rows of 128 B per instruction
            voff[i] = (uint32_t)(row * rs + (lane % 8) * 16);
        } else if (mode == 2) {
            voff[i] = (uint32_t)(q * 1024 + lane * 16);
        } else if (mode == 3) {
            voff[i] = (uint32_t)((size_t)blockIdx.x * STEP * 16 + q * 1024 + lane * 16);
        } else {
            const int row = (blockIdx.x * 64 + q * 8 + lane / 8) % 19200;
            voff[i] = (uint32_t)(row * 512 + (lane % 8) * 16);
        }
    }
    auto soff_of = [&](int k) -> uint32_t {
        if (mode <= 1) return (uint32_t)(((k + kstep0) % nk) * 128);
        if (mode == 2) return (uint32_t)((k % 64) * STEP);
        if (mode == 3) return (uint32_t)((k % 16) * STEP);
        return (uint32_t)((k % 4) * 128);
    };
    // prologue: S-1 steps in flight
    for (int s = 0; s < S - 1; ++s) {
#pragma unroll
        for (int i = 0; i < INS; ++i)
            bload16(voff[i], rsrc, soff_of(s), __builtin_amdgcn_readfirstlane(lbase + s * STEP + (i * NW + wave) * 1024));
    }
    float acc = 0.f;
    for (int k = 0; k < steps; ++k) {
        wait_vmcnt<INS * (S - 2)>();
        lds_barrier();
        const int nx = k + S - 1, buf = nx % S;
#pragma unroll
        for (int i = 0; i < INS; ++i)
            bload16(voff[i], rsrc, soff_of(nx), __builtin_amdgcn_readfirstlane(lbase + buf * STEP + (i * NW + wave) * 1024));
        acc += *reinterpret_cast<const float *>(lds + (k % S) * STEP + tid * 4);  // touch the landed buffer
    }
    wait_vmcnt<0>();
    if (acc == 12345.f) sink[blockIdx.x] = acc;
}

template <int STEP, int S, int NT>
void run(const char *src, uint32_t bytes, int mode, int wgs_per_cu, int rs, float *sink) {
    const int grid = 256 * wgs_per_cu, steps = 400;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto k = fill_kernel<STEP, S, NT>;
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k, dim3(grid), dim3(NT), 0, 0, src, bytes, mode, steps, rs, sink);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(NT), 0, 0, src, bytes, mode, steps, rs, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double per = ms / reps * 1e-3;
    const double bytes_cu = (double)STEP * (steps + S - 1) * wgs_per_cu;
    printf("{\"step_kb\": %d, \"stages\": %d, \"threads\": %d, \"mode\": %d, \"wg_per_cu\": %d, \"rs\": %d, \"us\": %.1f, "
           "\"gbs_per_cu\": %.1f, \"tbs_chip\": %.2f}\n",
           STEP / 1024, S, NT, mode, wgs_per_cu, rs, per * 1e6, bytes_cu / per / 1e9, bytes_cu * 256 / per / 1e12);
    fflush(stdout);
}

int main() {
    const size_t big = (size_t)1 << 30;
    char *src;
    float *sink;
    if (hipMalloc(&src, big) != hipSuccess || hipMalloc(&sink, 65536 * 4) != hipSuccess) return 1;
    hipMemset(src, 1, big);
    const uint32_t b32 = (uint32_t)(big - 4096);
    for (int mode : {0, 1, 2, 3, 4}) {
        for (int rs : {1536, 1664}) {
            if (mode > 1 && rs != 1536) continue;
            run<24576, 3, 256>(src, b32, mode, 2, rs, sink);
            run<24576, 3, 256>(src, b32, mode, 1, rs, sink);
            run<16384, 4, 256>(src, b32, mode, 2, rs, sink);
            run<32768, 2, 256>(src, b32, mode, 2, rs, sink);
            run<49152, 3, 512>(src, b32, mode, 1, rs, sink);
            run<65536, 2, 512>(src, b32, mode, 1, rs, sink);
            run<8192, 4, 256>(src, b32, mode, 4, rs, sink);
        }
    }
    return 0;
}
