// Second probe for the packed-fp32 fault: the faulting wgrad builds multiply the staged
// dY values by a PAIR of per-row masks {ym(row 2r), ym(row 2r+1)} that two v_cndmask_b32 write just
// before the packed multiply reads them as one 64-bit operand, e.g.
//     v_cndmask_b32_e64 v26, 0, 1.0, s[38:39]
//     v_cndmask_b32_e64 v27, 0, 1.0, s[34:35]
//     v_pk_mul_f32 v[54:55], v[10:11], v[26:27] op_sel:[0,1] op_sel_hi:[1,0]
// Replacing that multiply by a select made the same kernel exact (tools/gpu_r2d.sh, variant F); the
// isolated instruction forms with compiler-placed operands were exact (tools/pkfp32_probe.hip).  Here
// the sequence is written in inline asm with fixed registers, so the distance between the VGPR write
// and the packed read is controlled exactly:
//   W  writer of the mask register: 0 v_mov_b32, 1 v_cndmask_b32_e64 (vcc)
//   H  which half of the 64-bit operand was written last: 0 low dword, 1 high dword
//   F  form: 0 default (lo*lo, hi*hi), 1 op_sel:[0,1] op_sel_hi:[1,0] (lo*s.hi, hi*s.lo)
//   N  independent instructions (v_nop) between the write and the packed read: 0, 1, 2
// Each case runs in waves 0-3 of a 512-thread workgroup; waves 4-7 run MFMAs (mode 1) or the same
// checker (mode 3) or exit (mode 0).  Reports mismatching lane-iterations per case.
//
//   hipcc -O3 --offload-arch=gfx950 -o pkprobe2 tools/pkfp32_probe2.hip && ./pkprobe2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

#define NOPS0 ""
#define NOPS1 "v_nop\n\t"
#define NOPS2 "v_nop\n\tv_nop\n\t"
#define FORM0 ""
#define FORM1 " op_sel:[0,1] op_sel_hi:[1,0]"
// writers of v45 (high dword of v[44:45]) or v44 (low dword); the other dword is set earlier
#define WR0_H1 "v_mov_b32 v44, %[slo]\n\tv_mov_b32 v45, %[shi]\n\t"
#define WR0_H0 "v_mov_b32 v45, %[shi]\n\tv_mov_b32 v44, %[slo]\n\t"
#define WR1_H1 "v_mov_b32 v44, %[slo]\n\tv_cmp_lt_f32_e32 vcc, 0, %[shi]\n\tv_cndmask_b32_e64 v45, 0, 1.0, vcc\n\t"
#define WR1_H0 "v_mov_b32 v45, %[shi]\n\tv_cmp_lt_f32_e32 vcc, 0, %[slo]\n\tv_cndmask_b32_e64 v44, 0, 1.0, vcc\n\t"

#define CASE(W, H, F, N)                                                                                   \
    __device__ __forceinline__ void case_##W##H##F##N(float xlo, float xhi, float slo, float shi, float &r0, \
                                                        float &r1) {                                       \
        asm volatile("v_mov_b32 v40, %[xlo]\n\t"                                                            \
                     "v_mov_b32 v41, %[xhi]\n\t" WR##W##_H##H NOPS##N "v_pk_mul_f32 v[46:47], v[40:41], v[44:45]" \
                     FORM##F "\n\t"                                                                         \
                     "v_mov_b32 %[r0], v46\n\t"                                                             \
                     "v_mov_b32 %[r1], v47"                                                                 \
                     : [r0] "=v"(r0), [r1] "=v"(r1)                                                          \
                     : [xlo] "v"(xlo), [xhi] "v"(xhi), [slo] "v"(slo), [shi] "v"(shi)                       \
                     : "v40", "v41", "v44", "v45", "v46", "v47", "vcc");                                    \
    }

#define CASES_N(W, H, F) CASE(W, H, F, 0) CASE(W, H, F, 1) CASE(W, H, F, 2)
#define CASES_F(W, H) CASES_N(W, H, 0) CASES_N(W, H, 1)
CASES_F(0, 0)
CASES_F(0, 1)
CASES_F(1, 0)
CASES_F(1, 1)

constexpr int kCases = 24;

__device__ __forceinline__ float mask01(float v) { return v > 0.f ? 1.f : 0.f; }
__device__ __forceinline__ float s_mul(float a, float b) {  // scalar reference product (never packed)
    float r;
    asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ void checker(const float *in, int n, int iters, unsigned *bad) {
    const int lane = threadIdx.x & 63;
    unsigned cnt[kCases] = {};
    unsigned hist[kCases * 4] = {};  // (case, lane bit 4, element lo/hi)
    const int h = (lane >> 4) & 1;
    for (int it = 0; it < iters; ++it) {
        const int base = ((it * 97 + (blockIdx.x * 8 + (threadIdx.x >> 6)) * 131) % (n / 256)) * 256 + lane * 4;
        const float4 v = *reinterpret_cast<const float4 *>(in + base);
        const float xlo = v.x, xhi = v.y, slo = v.z, shi = v.w;
        int k = 0;
        float r0, r1;
        // expected products: writer 0 keeps (slo, shi); writer 1 turns the written dword into a 0/1 mask
#define RUN(W, H, F, N)                                                                                 \
    {                                                                                                   \
        case_##W##H##F##N(xlo, xhi, slo, shi, r0, r1);                                                  \
        const float sl = (W == 1 && H == 0) ? mask01(slo) : slo, sh = (W == 1 && H == 1) ? mask01(shi) : shi; \
        const float e0 = s_mul(xlo, F == 0 ? sl : sh), e1 = s_mul(xhi, F == 0 ? sh : sl);             \
        const bool b0 = __float_as_uint(r0) != __float_as_uint(e0), b1 = __float_as_uint(r1) != __float_as_uint(e1); \
        cnt[k] += b0 | b1;                                                                              \
        hist[4 * k + 2 * h] += b0;                                                                      \
        hist[4 * k + 2 * h + 1] += b1;                                                                  \
        ++k;                                                                                            \
    }
#define RUN_N(W, H, F) RUN(W, H, F, 0) RUN(W, H, F, 1) RUN(W, H, F, 2)
#define RUN_F(W, H) RUN_N(W, H, 0) RUN_N(W, H, 1)
        RUN_F(0, 0) RUN_F(0, 1) RUN_F(1, 0) RUN_F(1, 1)
    }
    for (int c = 0; c < kCases; ++c)
        if (cnt[c]) atomicAdd(&bad[c], cnt[c]);
    for (int c = 0; c < 4 * kCases; ++c)
        if (hist[c]) atomicAdd(&bad[kCases + c], hist[c]);
}

__global__ __launch_bounds__(512) void probe(const float *in, int n, int iters, int mode, unsigned *bad, float *sink) {
    const int wave = threadIdx.x >> 6;
    f32x16 acc;
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    if (wave < 4) {
        checker(in, n, iters, bad);
    } else if (mode == 1) {
        const bf16x8 a = {(__bf16)1.f, (__bf16)-1.f, (__bf16)0.5f, (__bf16)2.f, (__bf16)1.f, (__bf16)-1.f, (__bf16)0.25f, (__bf16)3.f};
        for (int it = 0; it < iters * 8; ++it) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, acc, 0, 0, 0);
    } else if (mode == 3) {
        checker(in, n, iters, bad);
    } else {
        return;
    }
    float t = 0.f;
    for (int i = 0; i < 16; ++i) t += acc[i];
    sink[blockIdx.x * 512 + threadIdx.x] = t;
}

int main(int argc, char **argv) {
    const int n = 1 << 22;
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    std::vector<float> h(n);
    uint32_t s = 12345;
    for (int i = 0; i < n; ++i) {
        s = s * 1664525u + 1013904223u;
        h[i] = ((int)(s >> 9) - (1 << 22)) * (1.0f / (1 << 20));
    }
    float *d_in, *d_sink;
    unsigned *d_bad;
    const int cus = 256;
    CHECK(hipMalloc(&d_in, n * sizeof(float)));
    CHECK(hipMalloc(&d_sink, (size_t)2 * cus * 512 * sizeof(float)));
    CHECK(hipMalloc(&d_bad, 5 * kCases * sizeof(unsigned)));
    CHECK(hipMemcpy(d_in, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
    const char *modes[] = {"checkers alone", "partner MFMA", "", "partner checker"};
    const int reps = argc > 2 ? atoi(argv[2]) : 1;
    for (int rep = 0; rep < reps; ++rep)
    for (int grid : {cus, 2 * cus}) {
        for (int mode : {0, 1}) {
            CHECK(hipMemset(d_bad, 0, 5 * kCases * sizeof(unsigned)));
            hipLaunchKernelGGL(probe, dim3(grid), dim3(512), 0, 0, d_in, n, iters, mode, d_bad, d_sink);
            CHECK(hipGetLastError());
            CHECK(hipDeviceSynchronize());
            unsigned b[5 * kCases];
            CHECK(hipMemcpy(b, d_bad, sizeof(b), hipMemcpyDeviceToHost));
            printf("grid %4d %-16s checks/case %.3g\n", grid, modes[mode], (double)grid * (mode == 3 ? 8 : 4) * 64 * iters);
            int k = 0;
            for (int W = 0; W < 2; ++W)
                for (int H = 0; H < 2; ++H)
                    for (int F = 0; F < 2; ++F) {
                        printf("   %-8s write %s form %-22s nops0..2:", W ? "cndmask" : "mov", H ? "hi" : "lo",
                               F ? "op_sel:[0,1],hi:[1,0]" : "default");
                        for (int N = 0; N < 3; ++N) printf(" %8u", b[k + N]);
                        printf("   [lanes&16==0 lo,hi | lanes&16 lo,hi]:");
                        for (int N = 0; N < 3; ++N)
                            printf(" %u,%u|%u,%u", b[kCases + 4 * (k + N)], b[kCases + 4 * (k + N) + 1],
                                   b[kCases + 4 * (k + N) + 2], b[kCases + 4 * (k + N) + 3]);
                        printf("\n");
                        k += 3;
                    }
            fflush(stdout);
        }
    }
    return 0;
}
