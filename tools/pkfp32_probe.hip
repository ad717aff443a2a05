// Probe for the packed-fp32 wrong-result fault seen in the bf16 wgrad.
//
// Hypothesis under test: a packed-fp32 VALU op (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32) returns a
// wrong element when ANOTHER wave on the same SIMD is executing MFMAs at the same time -- the wgrad
// faulted only when two workgroups shared a CU (two waves per SIMD, each mixing MFMA and v_pk_*), and
// was exact with one workgroup per CU (one wave per SIMD: its own MFMAs and VALU are issued in order).
//
// One 512-thread workgroup per CU: waves w and w+4 share a SIMD.  Waves 0-3 ("checkers") run a loop
// of packed-fp32 ops on known data, each checked bit for bit against the same arithmetic done with
// scalar v_mul_f32 / v_fma_f32 / v_add_f32 (all exact-IEEE fp32, so they must agree bitwise).  Waves
// 4-7 ("partners") run, by mode: 0 nothing (exit), 1 back-to-back bf16 MFMAs, 2 scalar VALU FMAs,
// 3 the same packed-fp32 checker loop, 4 MFMAs interleaved with packed ops in the CHECKER waves too.
// Output per mode: mismatches, and which (lane half, element) they hit.
//
//   hipcc -O3 --offload-arch=gfx950 -o pkprobe tools/pkfp32_probe.hip && ./pkprobe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

// the five operand-select forms hipcc emits for v_pk_mul_f32 (low result / high result):
//   F0 default                      x.lo*s.lo / x.hi*s.hi
//   F1 op_sel_hi:[1,0]              x.lo*s.lo / x.hi*s.lo   (current wgrad: broadcast of the row mask)
//   F2 op_sel_hi:[0,1]              x.lo*s.lo / x.lo*s.hi
//   F3 op_sel:[0,1] op_sel_hi:[1,0] x.lo*s.hi / x.hi*s.lo   (the faulting round-1 wgrad build)
//   F4 op_sel:[1,0] op_sel_hi:[0,1] x.hi*s.lo / x.lo*s.hi
template <int F>
__device__ __forceinline__ f32x2 pk_mul(f32x2 x, f32x2 s) {
    f32x2 r;
    if constexpr (F == 0) asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(s));
    if constexpr (F == 1) asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(x), "v"(s));
    if constexpr (F == 2) asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(x), "v"(s));
    if constexpr (F == 3) asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(r) : "v"(x), "v"(s));
    if constexpr (F == 4) asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(r) : "v"(x), "v"(s));
    return r;
}
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
    f32x2 r;
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ f32x2 pk_add(f32x2 a, f32x2 b) {
    f32x2 r;
    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float s_mul(float a, float b) {
    float r;
    asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float s_fma(float a, float b, float c) {
    float r;
    asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float s_add(float a, float b) {
    float r;
    asm volatile("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// bad[op] = mismatching lanes-iterations of op (0-4: v_pk_mul_f32 forms F0-F4, 5: v_pk_fma_f32,
// 6: v_pk_add_f32); bad[8 + 4*op + 2*half16 + elem]: histogram by (op, lane bit 4, element lo/hi)
constexpr int kOps = 7;
__device__ __forceinline__ void tally(int op, f32x2 got, float w0, float w1, int h, unsigned *cnt, unsigned *hist) {
    const bool e0 = __float_as_uint(got.x) != __float_as_uint(w0), e1 = __float_as_uint(got.y) != __float_as_uint(w1);
    cnt[op] += e0 | e1;
    hist[4 * op + 2 * h] += e0;
    hist[4 * op + 2 * h + 1] += e1;
}
__device__ void checker(const float *in, int n, int iters, unsigned *bad, bool with_mfma, f32x16 &acc) {
    const int lane = threadIdx.x & 63, h = (lane >> 4) & 1;
    unsigned cnt[kOps] = {};
    unsigned hist[4 * kOps] = {};
    const bf16x8 a = {(__bf16)1.f, (__bf16)2.f, (__bf16)3.f, (__bf16)4.f, (__bf16)5.f, (__bf16)6.f, (__bf16)7.f, (__bf16)8.f};
    for (int it = 0; it < iters; ++it) {
        const int base = ((it * 97 + (blockIdx.x * 8 + (threadIdx.x >> 6)) * 131) % (n / 256)) * 256 + lane * 4;
        const float4 v = *reinterpret_cast<const float4 *>(in + base);
        // the row-mask shape of the wgrad: s.lo / s.hi are 0/1 selects made right before the multiply
        const f32x2 x = {v.x, v.y}, s = {v.z > 0.f ? 1.f : 0.f, v.w > 0.f ? v.w : 0.f}, c = {v.w, v.x};
        if (with_mfma) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, acc, 0, 0, 0);
        const f32x2 p0 = pk_mul<0>(x, s), p1 = pk_mul<1>(x, s), p2 = pk_mul<2>(x, s), p3 = pk_mul<3>(x, s),
                    p4 = pk_mul<4>(x, s);
        if (with_mfma) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, acc, 0, 0, 0);
        const f32x2 pf = pk_fma(x, s, c);
        const f32x2 pa = pk_add(x, c);
        tally(0, p0, s_mul(x.x, s.x), s_mul(x.y, s.y), h, cnt, hist);
        tally(1, p1, s_mul(x.x, s.x), s_mul(x.y, s.x), h, cnt, hist);
        tally(2, p2, s_mul(x.x, s.x), s_mul(x.x, s.y), h, cnt, hist);
        tally(3, p3, s_mul(x.x, s.y), s_mul(x.y, s.x), h, cnt, hist);
        tally(4, p4, s_mul(x.y, s.x), s_mul(x.x, s.y), h, cnt, hist);
        tally(5, pf, s_fma(x.x, s.x, c.x), s_fma(x.y, s.y, c.y), h, cnt, hist);
        tally(6, pa, s_add(x.x, c.x), s_add(x.y, c.y), h, cnt, hist);
    }
    for (int op = 0; op < kOps; ++op)
        if (cnt[op]) atomicAdd(&bad[op], cnt[op]);
    for (int i = 0; i < 4 * kOps; ++i)
        if (hist[i]) atomicAdd(&bad[8 + i], hist[i]);
}

__global__ __launch_bounds__(512) void probe(const float *in, int n, int iters, int mode, unsigned *bad, float *sink) {
    const int wave = threadIdx.x >> 6;
    f32x16 acc;
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    if (wave < 4) {
        checker(in, n, iters, bad, mode == 4, acc);
    } else {
        if (mode == 0) return;
        if (mode == 1 || mode == 4) {
            const bf16x8 a = {(__bf16)1.f, (__bf16)-1.f, (__bf16)0.5f, (__bf16)2.f, (__bf16)1.f, (__bf16)-1.f, (__bf16)0.25f, (__bf16)3.f};
            for (int it = 0; it < iters * 4; ++it) {
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, acc, 0, 0, 0);
            }
        } else if (mode == 2) {
            float x = in[threadIdx.x], y = 1.0001f;
            for (int it = 0; it < iters * 16; ++it) x = s_fma(x, y, 0.5f);
            acc[0] = x;
        } else if (mode == 3) {
            checker(in, n, iters, bad, false, acc);
        }
    }
    float t = 0.f;
    for (int i = 0; i < 16; ++i) t += acc[i];
    sink[blockIdx.x * 512 + threadIdx.x] = t;
}

int main(int argc, char **argv) {
    const int n = 1 << 22;
    const int iters = argc > 1 ? atoi(argv[1]) : 4000;
    std::vector<float> h(n);
    uint32_t s = 12345;
    for (int i = 0; i < n; ++i) {
        s = s * 1664525u + 1013904223u;
        h[i] = ((int)(s >> 9) - (1 << 22)) * (1.0f / (1 << 20));
    }
    float *d_in, *d_sink;
    unsigned *d_bad;
    int cus = 256;
    const int blocks = cus * 2;  // 2 x 512-thread workgroups per CU = 4 waves per SIMD
    CHECK(hipMalloc(&d_in, n * sizeof(float)));
    CHECK(hipMalloc(&d_sink, (size_t)blocks * 512 * sizeof(float)));
    CHECK(hipMalloc(&d_bad, 64 * sizeof(unsigned)));
    CHECK(hipMemcpy(d_in, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
    const char *opn[kOps] = {"mulF0", "mulF1", "mulF2", "mulF3", "mulF4", "fma", "add"};
    const char *names[] = {"checkers alone", "partner MFMA loop", "partner scalar VALU", "partner packed-fp32",
                           "checkers interleave MFMA + partner MFMA"};
    for (int grid : {cus, blocks}) {
        for (int mode = 0; mode < 5; ++mode) {
            CHECK(hipMemset(d_bad, 0, 64 * sizeof(unsigned)));
            hipLaunchKernelGGL(probe, dim3(grid), dim3(512), 0, 0, d_in, n, iters, mode, d_bad, d_sink);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            unsigned b[64];
            CHECK(hipMemcpy(b, d_bad, sizeof(b), hipMemcpyDeviceToHost));
            const double checks = (double)grid * (mode == 3 ? 8 : 4) * 64 * iters;
            printf("grid %4d mode %d %-42s checks/op %.3g  bad:", grid, mode, names[mode], checks);
            for (int op = 0; op < kOps; ++op) printf(" %s=%u", opn[op], b[op]);
            printf("\n");
            for (int op = 0; op < kOps; ++op)
                if (b[op])
                    printf("    %s: lanes&16==0 lo %u hi %u | lanes&16 lo %u hi %u\n", opn[op], b[8 + 4 * op], b[9 + 4 * op],
                           b[10 + 4 * op], b[11 + 4 * op]);
            fflush(stdout);
        }
    }
    return 0;
}
