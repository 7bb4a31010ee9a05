// plan_kernels.hpp — device helpers shared by the BSMR plan kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace bsmr {
namespace dev {

using u32 = uint32_t;
using u64 = uint64_t;

constexpr u32 ASSIGNED = 0x80000000u;  // cluster-state word: bit 31 = assigned, low bits = id
constexpr u32 ST_NONE = 0xFFFFFFFFu;   // start word: cluster does not exist

// Relaxed agent-scope atomics on global memory (global_load/store ... sc1): the hand-off words
// of the clustering chain are single 4-byte granules, so no payload fence is needed
// (cdna_hip_programming.md §6 Guideline 16, R2).
__device__ __forceinline__ u32 ld_agent(const u32* p) {
    return __hip_atomic_load(const_cast<u32*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(u32* p, u32 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ u32 lane_id() { return __lane_id(); }

// clustering candidate filter (cluster_filter.hip): row q of the bit triangle holds the 32-bit
// words [q / 32, W) of positions p, so it starts at sum_{r < q} (W - r / 32)
__host__ __device__ __forceinline__ u64 fbits_row_offset(u32 q, u32 W) {
    const u64 a = q >> 5, b = q & 31;
    return static_cast<u64>(q) * W - (16 * a * (a - 1) + a * b);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// inclusive prefix sum across the 64 lanes of a wave
__device__ __forceinline__ u32 wave_incl_scan(u32 v) {
    const u32 l = __lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u32 t = __shfl_up(v, o);
        if (l >= static_cast<u32>(o)) v += t;
    }
    return v;
}

}  // namespace dev
}  // namespace bsmr
