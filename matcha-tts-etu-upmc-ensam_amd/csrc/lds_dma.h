// LDS-DMA primitives shared by the GEMM (conv_gemm_glds.hip) and attention (attention.hip) kernels:
// global / buffer loads that write LDS directly (no VGPR round trip), and counted vmcnt waits.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mtts {

// One global_load_lds_dwordx4: 16 bytes per lane from `src` into LDS at lds_base + 16*lane.  Issued as
// inline asm so hipcc's waitcnt pass does not see an LDS write it cannot disambiguate from the
// fragment reads of the other stages (it inserted vmcnt(0) before them, draining every prefetch);
// the kernel orders each buffer itself with counted vmcnt waits and barriers.  M0 holds the LDS base.
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

// One buffer_load_dwordx4 ... lds: 16 bytes per lane from rsrc + voff + soff into LDS at lds_base + 16*lane.
// A lane whose voff lies past the descriptor's num_records reads zeros (masked / out-of-range rows:
// kDmaOob); a per-step advance can live in the scalar soff, so a loop issues its loads with no vector
// address arithmetic.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kDmaOob = 0x80000000u;

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

// One buffer_load_dword ... lds: 4 bytes per lane into LDS at lds_base + 4*lane (per-element bounds: a lane
// whose voff lies past num_records reads a zero)
__device__ __forceinline__ void bload4(uint32_t voff, u32x4 rsrc, uint32_t soff, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %4\n\t"
        "s_nop 0\n\t"
        "buffer_load_dword %1, %2, %3 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
        : "memory");
}

// LDS byte address of a __shared__ pointer, wave-uniform (the M0 operand of the DMA loads)
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void *)p);
}

// s_waitcnt vmcnt(N) (expcnt / lgkmcnt left at their maxima; gfx9 encoding: vmcnt[3:0] | [15:14])
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

}  // namespace mtts
