// LDS helpers shared by the MFMA kernels (gfx950).
//
// hipcc's waitcnt pass cannot prove that a ds_read does not alias an in-flight
// global_load_lds (LDS-DMA) and drains it with s_waitcnt vmcnt(0) before the
// read, which serialises the next tile's prefetch with the current tile's math.
// Fragment reads are therefore issued as inline asm (invisible to that pass);
// the caller waits with lds_wait_all() — an explicit lgkmcnt(0) followed by a
// sched_barrier so no register-only MFMA is hoisted above it (guide §5.7
// item 1, §5.4 rule 18).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace acemi {

typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ uint32_t lds_addr(const void* generic_lds_ptr) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)generic_lds_ptr;
}

template <int OFF>
__device__ __forceinline__ uint4 ds_read_b128_at(uint32_t addr) {
    u32x4_t v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
    return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ uint4 ds_read_b128_v(uint32_t addr) {
    u32x4_t v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
    return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ void lds_wait_all() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// s_waitcnt vmcnt(N), N compile-time (lgkmcnt / expcnt untouched)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

}  // namespace acemi
