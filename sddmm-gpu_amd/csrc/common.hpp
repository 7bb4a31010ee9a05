// common.hpp — shared constants, error plumbing and a small RAII device buffer.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "bsmr.h"

namespace bsmr {

using u32 = uint32_t;
using u64 = uint64_t;

// Reference tile constants (include/BSMR.hpp:8-10, include/TensorCoreConfig.cuh:11-14,
// include/sddmmKernel.cuh:11-17). They define the plan layout, so they are part of the boundary.
constexpr u32 NULLV = 0xFFFFFFFFu;
constexpr u32 PANEL = 16;            // ROW_PANEL_SIZE
constexpr u32 BCOL = 16;             // BLOCK_COL_SIZE
constexpr u32 TILE = PANEL * BCOL;   // BLOCK_SIZE
constexpr u32 REF_DENSE_BLOCKS_PER_TB = 4;
constexpr u32 REF_SPARSE_DATA_PER_TB = 128;
constexpr u32 REF_MAX_SHMEM = 49152;  // maxSharedMemoryPerBlock, calculateBlockSize input

void set_error(const std::string& msg);
const char* get_error();

// Turn a HIP failure into a status + message (never throws).
#define BSMR_HIP(expr)                                                                      \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            ::bsmr::set_error(std::string(#expr) + ": " + hipGetErrorString(e_) + " (" +    \
                              __FILE__ + ":" + std::to_string(__LINE__) + ")");             \
            return BSMR_ERR_HIP;                                                            \
        }                                                                                   \
    } while (0)

#define BSMR_CHECK(expr)                       \
    do {                                       \
        int s_ = (expr);                       \
        if (s_ != BSMR_OK) return s_;          \
    } while (0)

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    int alloc(size_t count) {
        release();
        n = count;
        if (count == 0) return BSMR_OK;
        BSMR_HIP(hipMalloc(&p, count * sizeof(T)));
        return BSMR_OK;
    }
    int upload(const T* h, size_t count, hipStream_t s) {
        BSMR_CHECK(alloc(count));
        if (count && h) BSMR_HIP(hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s));
        return BSMR_OK;
    }
    int download(std::vector<T>& h, hipStream_t s) const {
        h.resize(n);
        if (n) {
            BSMR_HIP(hipMemcpyAsync(h.data(), p, n * sizeof(T), hipMemcpyDeviceToHost, s));
            BSMR_HIP(hipStreamSynchronize(s));
        }
        return BSMR_OK;
    }
    T* data() const { return p; }
    size_t size() const { return n; }
};

}  // namespace bsmr
